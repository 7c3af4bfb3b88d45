#!/bin/bash
# Round-6: prefetch A/B after the scalar run loads, then the UInt8 gather counter passes at the
# default knobs.  Output: gpurun_out/r6c/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --only gatherp --reps 10 > $O/gatherp.log 2>&1 || { tail $O/gatherp.log; exit 1; }
grep '^{' $O/gatherp.log | cut -c1-150
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" bash scripts/gpu_pmc_groups.sh r6c u8gather > $O/pmc.out 2>&1 || { tail $O/pmc.out; exit 1; }
cut -c1-200 $O/u8gather.pmc.jsonl
echo done
