#!/bin/bash
# Round 5: occupancy sweep of the one-row pointwise kernel (bench_configs group rowlds).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 500 python3 tools/bench_configs.py --only rowlds --reps 10 > $O/rowlds.log 2>&1 || { tail -20 $O/rowlds.log; exit 1; }
grep -c '^{' $O/rowlds.log
