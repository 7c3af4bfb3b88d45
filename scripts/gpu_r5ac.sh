#!/bin/bash
# Round 5: the whole tree with the UInt16 gather prefetch default -- smoke, GPU suite, bench,
# then the prefetch A/B once more.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/gpu_r5check.sh || exit 1
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only gatherp --reps 10 > $O/gatherp.log 2>&1 || { tail -20 $O/gatherp.log; exit 1; }
grep '^{' $O/gatherp.log | cut -c1-150
