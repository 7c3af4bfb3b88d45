#!/bin/bash
# One tools/bench_configs.py group on the GPU (in-process A/B or timing rows), optionally after a
# focused pytest selection.  Output: gpurun_out/<out>/.
#   bash scripts/gpu_ab.sh <out> <group> ["<pytest args>"]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; G=$2; mkdir -p $O
if [ -n "${3:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $3 > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 tools/bench_configs.py --only $G --reps 10 > $O/$G.log 2>&1 || { tail $O/$G.log; exit 1; }
grep '^{' $O/$G.log | cut -c1-170
echo done
