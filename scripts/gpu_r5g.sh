#!/bin/bash
# Round 5: row-kernel A/B + parity of the pointwise tests + bench; UInt8 calibration counters;
# then the VMM probe through libvolkit (last: it may crash the HIP runtime).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py --only rowk --reps 10 > $O/rowk.log 2>&1 || { tail -20 $O/rowk.log; exit 1; }
grep '^{' $O/rowk.log | cut -c1-140
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_general.py tests/test_gpu_configs.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pw.log 2>&1 || { tail -40 $O/pytest_pw.log; exit 1; }
tail -2 $O/pytest_pw.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
bash scripts/gpu_r5e.sh > $O/u8cal.out 2>&1 || { tail -20 $O/u8cal.out; exit 1; }
tail -30 $O/u8cal.out | cut -c1-400
timeout -k 10 120 python -u tools/vmm_probe.py lib torch > $O/vmm_lib.log 2>&1 || { echo "vmm lib rc=$?"; tail -30 $O/vmm_lib.log; exit 1; }
tail -14 $O/vmm_lib.log
