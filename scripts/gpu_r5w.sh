#!/bin/bash
# Round 5: row copy of small bricks with halos (knob decompose.rows) -- parity, then the A/B.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decompose.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 tools/bench_configs.py --only decrows --reps 10 > $O/decrows.log 2>&1 || { tail -20 $O/decrows.log; exit 1; }
grep '^{' $O/decrows.log | cut -c1-200
