#!/bin/bash
# Round 5: UInt8 FETCH calibration and whole-volume UInt8 vs UInt16 counters (tools/bench_configs.py
# group u8cal): event timings, then read requests by size (32/64/128 B), FETCH_SIZE, WRITE_SIZE +
# DRAM reads, and an SQ pass, per dispatch.
set -u
cd "$(dirname "$0")/.."
export PMC_PASSES="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;FETCH_SIZE;WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
bash scripts/gpu_pmc_groups.sh r5e u8cal
