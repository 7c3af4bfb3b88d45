#!/bin/bash
# BrickDecompose small-brick counters.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4i}
PMC_KERNEL=brickCopyKernel PMC_EXTRA="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
  bash scripts/gpu_pmc_groups.sh $O dec16 || exit 1
