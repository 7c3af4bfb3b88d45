#!/bin/bash
# Round 5: the 2048^3 placement states with counters (tools/placement_pmc.py): one process per
# pass, each pass's allocations joined with its own timings.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
PASSES=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum"
        "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
        "FETCH_SIZE GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
        "WRITE_SIZE TCC_EA0_RDREQ_sum")
timeout -k 10 240 python3 tools/placement_pmc.py > $O/plain.log 2>&1 || { tail -20 $O/plain.log; exit 1; }
cat $O/plain.log
i=0
for pass in "${PASSES[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $O/p$i/p0 -o run --output-format csv -- python3 tools/placement_pmc.py > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  python3 scripts/pmc_dispatch.py $O/p$i $O/p$i.log 4 pointwiseVec > $O/p$i.jsonl && cat $O/p$i.jsonl
  i=$((i+1))
done
