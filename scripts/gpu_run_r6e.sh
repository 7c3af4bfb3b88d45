#!/bin/bash
# Round-6: row-image BrickDecompose (parity, A/B).  Output: gpurun_out/r6e/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_decompose.py -m gpu -k "row_image" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only decrow --reps 10 > $O/decrow.log 2>&1 || { tail $O/decrow.log; exit 1; }
grep '^{' $O/decrow.log | cut -c1-170
echo done
