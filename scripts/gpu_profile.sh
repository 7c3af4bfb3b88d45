#!/bin/bash
# rocprofv3 evidence for the bench: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in
# separate PMC passes (TCC slots: FETCH_SIZE 3, WRITE_SIZE 2 -> cannot share a pass).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
python3 scripts/parse_pmc.py $OUT 1024 > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
grep '^{' $OUT/trace.log | tail -1
