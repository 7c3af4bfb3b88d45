#!/bin/bash
# Round 5: the whole tree with non-16-B source rows staged in the LDS gather -- smoke, GPU suite,
# bench, then the A/B (knob resample.any_rows).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/gpu_r5check.sh || exit 1
O=gpurun_out/r5ad
mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only gathera --reps 10 > $O/gathera.log 2>&1 || { tail -20 $O/gathera.log; exit 1; }
grep '^{' $O/gathera.log | cut -c1-150
