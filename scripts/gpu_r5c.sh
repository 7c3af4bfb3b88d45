#!/bin/bash
# Round 5: the HIP-only VMM probe with copies from an offset inside the mapping.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 60 python -u tools/vmm_probe.py fresh > $O/vmm_fresh.log 2>&1 || { echo "vmm fresh rc=$?"; tail -30 $O/vmm_fresh.log; exit 1; }
tail -3 $O/vmm_fresh.log
timeout -k 10 60 python -u tools/vmm_probe.py reuse > $O/vmm_reuse.log 2>&1 || { echo "vmm reuse rc=$?"; tail -30 $O/vmm_reuse.log; exit 1; }
tail -3 $O/vmm_reuse.log
