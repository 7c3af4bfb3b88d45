#!/bin/bash
# pointwise parity + sub-box PMC (FETCH_SIZE / WRITE_SIZE) + weak spots.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-subbox}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python3 tools/bench_configs.py --only subbox --reps 5"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 scripts/parse_pmc.py $O 0 > $O/pmc_summary.json && grep -A5 "pointwiseVec" $O/pmc_summary.json
grep '^{' $O/trace.log
timeout -k 10 300 python3 tools/bench_configs.py --only weakspots --reps 10 > $O/weak.log 2>&1 || { tail -20 $O/weak.log; exit 1; }
grep '^{' $O/weak.log
