#!/bin/bash
# Development loop on the GPU box: a pytest selection, then a tools/bench_configs.py group,
# then (PROF=1) the same group under rocprofv3 --kernel-trace --stats.
#   [PROF=1] bash scripts/gpu_dev.sh "<pytest -k expr>" "<bench_configs --only group>"
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-}; G=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/dev_pytest.log 2>&1
  rc=$?; tail -n 4 gpurun_out/dev_pytest.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/dev_pytest.log; exit $rc; }
fi
[ -z "$G" ] && exit 0
timeout -k 10 400 python tools/bench_configs.py --only "$G" > gpurun_out/dev_bench.log 2>&1 || { tail -30 gpurun_out/dev_bench.log; exit 1; }
grep '^{' gpurun_out/dev_bench.log
[ "${PROF:-0}" = 1 ] || exit 0
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/devprof -o run --output-format csv -- python3 tools/bench_configs.py --only "$G" --reps 3 > gpurun_out/dev_prof.log 2>&1 || { tail -30 gpurun_out/dev_prof.log; exit 1; }
f=$(find gpurun_out/devprof -name "run_kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | cut -c1-220
