#!/bin/bash
# Round 5: UInt16 row-kernel occupancy A/B, then the 2048^3 placement-state counters (r5f).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only u16row --reps 10 > $O/u16row.log 2>&1 || { tail -20 $O/u16row.log; exit 1; }
grep -c '^{' $O/u16row.log
bash scripts/gpu_r5f.sh
