#!/bin/bash
# Round 5: histogram tiles side by side (knob histogram.pair_tiles) -- parity, then the A/B.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_reduce.py -m gpu -x -q --timeout 120 --timeout-method thread -k "histogram" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/bench_configs.py --only pairtiles --reps 10 > $O/pairtiles.log 2>&1 || { tail -20 $O/pairtiles.log; exit 1; }
grep '^{' $O/pairtiles.log | cut -c1-200
