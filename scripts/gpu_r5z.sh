#!/bin/bash
# Round 5: counters of the staged brick copy, UInt8 / UInt16 16^3 + halo 1, aligned_lds 0 / 4 / 3.
set -u
cd "$(dirname "$0")/.."
export PMC_KERNEL=brickCopyKernel
export PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
bash scripts/gpu_pmc_groups.sh r5z decedge
