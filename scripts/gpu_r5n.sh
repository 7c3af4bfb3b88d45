#!/bin/bash
# Round 5: XCD mapping A/B of the row kernel (group rowswz) + row-kernel parity with it.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 400 python3 tools/bench_configs.py --only rowswz --reps 10 > $O/rowswz.log 2>&1 || { tail -20 $O/rowswz.log; exit 1; }
grep -c '^{' $O/rowswz.log
