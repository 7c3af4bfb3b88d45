#!/bin/bash
# Round-4 counters: Float32 phase-shifted / UInt8 x0=100 pointwise (f32shift) and the P16 histogram
# (p16) with an LDS pass.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4b}
PMC_EXTRA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
  bash scripts/gpu_pmc_groups.sh $O p16 || exit 1
bash scripts/gpu_pmc_groups.sh $O f32shift || exit 1
mkdir -p gpurun_out/$O
timeout -k 10 600 python3 tools/bench_configs.py --only f32dw --reps 10 > gpurun_out/$O/f32dw.bench.log 2>&1 || { tail -20 gpurun_out/$O/f32dw.bench.log; exit 1; }
grep '^{' gpurun_out/$O/f32dw.bench.log
