#!/bin/bash
# Round 5: edge mode of the staged brick copy (knob decompose.aligned_lds 4) -- parity, then the A/B.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decompose.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 tools/bench_configs.py --only decedge --reps 10 > $O/decedge.log 2>&1 || { tail -20 $O/decedge.log; exit 1; }
grep '^{' $O/decedge.log | cut -c1-200
