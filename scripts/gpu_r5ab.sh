#!/bin/bash
# Round 5: next-row prefetch of the LDS gather (knob resample.prefetch) -- parity, then A/B.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resample_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 tools/bench_configs.py --only gatherp --reps 10 > $O/gatherp.log 2>&1 || { tail -20 $O/gatherp.log; exit 1; }
grep '^{' $O/gatherp.log | cut -c1-170
