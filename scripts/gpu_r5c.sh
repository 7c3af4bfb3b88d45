#!/bin/bash
# Round 5: the VMM probe through libvolkit (arena chunk released, mapping at its VA, library
# kernels and vktHipMemcpy on the mapping) under PyTorch's HIP runtime.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 120 python -u tools/vmm_probe.py lib torch > $O/vmm_lib.log 2>&1 || { echo "vmm lib rc=$?"; tail -30 $O/vmm_lib.log; exit 1; }
tail -14 $O/vmm_lib.log
