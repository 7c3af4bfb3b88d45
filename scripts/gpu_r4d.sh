#!/bin/bash
# Round-4: integer moments with branch-free per-step extremes; variants A/B + counters.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4d}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest tests/test_reduce.py tests/test_gpu_multirank.py tests/test_slab_reduce_gloo.py \
   -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -3 gpurun_out/$O/pytest.log
timeout -k 10 600 python3 tools/bench_configs.py --only mompipe --reps 10 > gpurun_out/$O/mompipe.bench.log 2>&1 || { tail -20 gpurun_out/$O/mompipe.bench.log; exit 1; }
grep '^{' gpurun_out/$O/mompipe.bench.log
timeout -k 10 600 python3 tools/bench_configs.py --only momf --reps 10 > gpurun_out/$O/momf.bench.log 2>&1 || { tail -20 gpurun_out/$O/momf.bench.log; exit 1; }
grep '^{' gpurun_out/$O/momf.bench.log
PMC_KERNEL=aggregatesMomentsU16Kernel PMC_EXTRA="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES" \
  bash scripts/gpu_pmc_groups.sh $O mom1 || exit 1
