#!/bin/bash
# Round-4: 4-GiB Float32 operands on the 32-bit general path, masked / pipelined integer moments,
# BrickDecompose batching A/B.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r4c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_reduce.py tests/test_gpu_general.py tests/test_decompose.py \
   "tests/test_gpu_large.py::test_float32_4gib_operands_shifted_parity" \
   -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for g in mompipe f32shift decbatch; do
  timeout -k 10 600 python3 tools/bench_configs.py --only $g --reps 10 > $O/$g.bench.log 2>&1 || { tail -20 $O/$g.bench.log; exit 1; }
  grep '^{' $O/$g.bench.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mompipe_trace -o run --output-format csv -- \
  python3 tools/bench_configs.py --only mompipe --reps 5 > $O/mompipe_trace.log 2>&1 || { tail -20 $O/mompipe_trace.log; exit 1; }
find $O/mompipe_trace -name "*kernel_stats.csv" -exec cp {} $O/mompipe_kernel_stats.csv \;
grep -i "moment" $O/mompipe_kernel_stats.csv | cut -c1-300
