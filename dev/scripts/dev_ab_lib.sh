#!/bin/bash
# A/B of two libvolkit builds in alternating processes on one box (VOLKIT_LIB override):
#   bash scripts/dev_ab_lib.sh <old.so> <group> [rounds]
set -u
cd "$(dirname "$0")/.."
OLD=$1; G=$2; N=${3:-2}
for r in $(seq 1 $N); do
  for lib in "$OLD" volkit_amd/lib/libvolkit.so; do
    echo "== round $r lib $lib"
    VOLKIT_LIB=$(realpath $lib) timeout -k 10 120 python3 tools/bench_configs.py --only "$G" 2>&1 | grep '^{' | cut -c1-120 || exit 1
  done
done
