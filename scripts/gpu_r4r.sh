#!/bin/bash
# Unified store statements in the pointwise kernels: parity, then f32shift timings + counters.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4r}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -40 gpurun_out/$O/pytest.log; exit 1; }
tail -2 gpurun_out/$O/pytest.log
bash scripts/gpu_pmc_groups.sh $O f32shift || exit 1
