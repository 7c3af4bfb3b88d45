#!/bin/bash
# Round 5: MODE-1 rows kernel parity + sub-box A/B (group rowsk).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_general.py -k "rows_kernel or row_kernel" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python3 tools/bench_configs.py --only rowsk --reps 10 > $O/rowsk.log 2>&1 || { tail -20 $O/rowsk.log; exit 1; }
grep -c '^{' $O/rowsk.log
