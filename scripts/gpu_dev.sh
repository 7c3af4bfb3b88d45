#!/bin/bash
# Development loop on the GPU box: a pytest selection, then tools/bench_configs.py cases.
#   bash scripts/gpu_dev.sh "<pytest -k expr>" "<bench_configs --only group>" [pytest files]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-}
ONLY=${2:-}
FILES=${3:-tests}
if [ -n "$K" ]; then
    timeout -k 10 900 python -m pytest $FILES -m gpu -q -x -k "$K" > gpurun_out/dev_pytest.log 2>&1
    rc=$?; tail -n 25 gpurun_out/dev_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$ONLY" ]; then
    timeout -k 10 600 python tools/bench_configs.py --only "$ONLY" > gpurun_out/dev_bench.log 2>&1
    rc=$?; grep '^{' gpurun_out/dev_bench.log || tail -20 gpurun_out/dev_bench.log; exit $rc
fi
exit 0
