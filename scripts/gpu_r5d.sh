#!/bin/bash
# Round 5: comm watcher + overlapped slab resample tests, the whole GPU suite, then the VMM probe
# through libvolkit (last: it may crash the HIP runtime).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_comm.py tests/test_gpu_slab_range.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/comm.log 2>&1 || { tail -60 $O/comm.log; exit 1; }
grep -a "passed\|failed\|skipped" $O/comm.log | tail -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u tools/vmm_probe.py lib torch > $O/vmm_lib.log 2>&1 || { echo "vmm lib rc=$?"; tail -30 $O/vmm_lib.log; exit 1; }
tail -12 $O/vmm_lib.log
