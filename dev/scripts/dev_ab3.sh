#!/bin/bash
# Alternating A/B/C runs of the 'metric' bench_configs group with three library builds.
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for v in old D; do
    echo "== round $r $v"
    VOLKIT_LIB=$(realpath abtmp/libvolkit_$v.so) timeout -k 10 120 python3 tools/bench_configs.py --only metric 2>&1 | grep '^{' | grep -v Resample | cut -c1-110 || exit 1
  done
done
