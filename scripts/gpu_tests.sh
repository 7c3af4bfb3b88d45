#!/bin/bash
# Selected GPU test files (bounded), then optional bench_configs groups.  Output: gpurun_out/$1/.
#   bash scripts/gpu_tests.sh <outdir> "<test files>" [groups...]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
T=$1; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for g in "$@"; do
  timeout -k 10 600 python3 tools/bench_configs.py --only $g --reps 10 > $O/$g.bench.log 2>&1 || { tail -20 $O/$g.bench.log; exit 1; }
  grep '^{' $O/$g.bench.log
done
