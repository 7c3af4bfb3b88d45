#!/bin/bash
# pointwise engine: parity tests + weak-spot timings.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-pw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_reference_kat.py tests/test_decompose.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 tools/bench_configs.py --only weakspots --reps 10 > $O/weak.log 2>&1 || { tail -20 $O/weak.log; exit 1; }
grep '^{' $O/weak.log
