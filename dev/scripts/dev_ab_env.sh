#!/bin/bash
# Alternating-process A/B of an environment knob: bash scripts/dev_ab_env.sh VAR "v1 v2" group [rounds]
set -u
cd "$(dirname "$0")/.."
VAR=$1; VALS=$2; G=$3; N=${4:-2}
for r in $(seq 1 $N); do
  for v in $VALS; do
    echo "== round $r $VAR=$v"
    env $VAR=$v timeout -k 10 150 python3 tools/bench_configs.py --only "$G" 2>&1 | grep '^{' | cut -c1-110 || exit 1
  done
done
