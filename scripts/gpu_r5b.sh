#!/bin/bash
# Round 5: the arena-release test, the whole GPU suite, the default bench, then the VMM probe
# without libvolkit (fresh VA, then reused VA) -- last, since it may crash the HIP runtime.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_memset.py -k "arena" -x -v -s --timeout 120 --timeout-method thread > $O/arena.log 2>&1 || { tail -40 $O/arena.log; exit 1; }
grep -a "VA reused\|passed\|failed" $O/arena.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 60 python -u tools/vmm_probe.py fresh > $O/vmm_fresh.log 2>&1 || { echo "vmm fresh rc=$?"; tail -30 $O/vmm_fresh.log; exit 1; }
tail -3 $O/vmm_fresh.log
timeout -k 10 60 python -u tools/vmm_probe.py reuse > $O/vmm_reuse.log 2>&1 || { echo "vmm reuse rc=$?"; tail -30 $O/vmm_reuse.log; exit 1; }
tail -3 $O/vmm_reuse.log
