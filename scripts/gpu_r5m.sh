#!/bin/bash
# Round 5: Float32 3-stream shifted SumRange counters (group f32s3), config 2 timings.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
export PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
bash scripts/gpu_pmc_groups.sh r5m f32s3 > gpurun_out/r5m_f32s3.out 2>&1 || { tail -20 gpurun_out/r5m_f32s3.out; exit 1; }
cat gpurun_out/r5m_f32s3.out | cut -c1-300
timeout -k 10 300 python3 tools/bench_configs.py --only config2 --reps 20 > gpurun_out/r5m/config2.log 2>&1 || { tail -20 gpurun_out/r5m/config2.log; exit 1; }
grep '^{' gpurun_out/r5m/config2.log
