#!/bin/bash
# Round-6 development run: the loader-wave gather (parity, A/B).  Output: gpurun_out/r6b/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resample_fuzz.py -k "rows_per_wave or padded" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only rpwab --reps 10 > $O/rpwab.log 2>&1 || { tail $O/rpwab.log; exit 1; }
grep '^{' $O/rpwab.log | cut -c1-150
echo done
