#!/bin/bash
# Alternating-process A/B of an environment knob on bench.py (N=1) and the 2048^3 size point.
set -u
cd "$(dirname "$0")/.."
VAR=$1; VALS=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for v in $VALS; do
    echo "== round $r $VAR=$v"
    env $VAR=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-copy-peak --steps 30 --warmup 20 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels_ms'])" || exit 1
    env $VAR=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-copy-peak --steps 10 --warmup 5 --dst 2048 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('2048^3', d['value'], d['kernels_ms'])" || exit 1
  done
done
