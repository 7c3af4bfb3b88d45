#!/bin/bash
# Round 5: occupancy cap sweep for the UInt8 row / rows kernels.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only rowslds --reps 20 > $O/rowslds.log 2>&1 || { tail -20 $O/rowslds.log; exit 1; }
grep '^{' $O/rowslds.log | cut -c1-170
