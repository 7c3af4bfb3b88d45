#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) over one tools/bench_configs.py group.
#   bash scripts/gpu_pmc_group.sh <group> <outdir>
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
G=$1; OUT=gpurun_out/$2
mkdir -p $OUT
B="python3 tools/bench_configs.py --only $G --reps 2"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
python3 scripts/parse_pmc.py $OUT 0 > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
