#!/bin/bash
# Round 5: Transform vector-kernel shapes (knob transform.shape) -- parity, then the A/B.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_transform_device.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/bench_configs.py --only tshape --reps 20 > $O/tshape.log 2>&1 || { tail -20 $O/tshape.log; exit 1; }
grep '^{' $O/tshape.log | cut -c1-220
