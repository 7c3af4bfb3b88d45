#!/bin/bash
# weak-spot kernels: kernel trace + FETCH_SIZE + WRITE_SIZE passes.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-weak}
mkdir -p $O
B="python3 tools/bench_configs.py --only weakspots --reps 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep '^{' $O/trace.log
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
python3 scripts/parse_pmc.py $O 0 > $O/pmc_summary.json && cat $O/pmc_summary.json
