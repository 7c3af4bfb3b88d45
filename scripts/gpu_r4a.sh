#!/bin/bash
# Round-4 checks: aggregates moments, allocator, context, comm tests; then the moments bench group.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r4a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_reduce.py tests/test_memset.py tests/test_hip_context.py tests/test_comm.py tests/test_decompose.py tests/test_gpu_multirank.py tests/test_gpu_slab_range.py tests/test_gpu_general.py \
   -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for g in moments decblk; do
  timeout -k 10 600 python3 tools/bench_configs.py --only $g --reps 10 > $O/$g.bench.log 2>&1 || { tail -20 $O/$g.bench.log; exit 1; }
  grep '^{' $O/$g.bench.log
done
