#!/bin/bash
# Round-4: BrickDecompose kernel times (kernel trace of the decbatch group), arena steadiness over
# re-allocations of the library's own volumes at 1024^3 and 2048^3.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4f}
mkdir -p gpurun_out/$O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$O/dec_trace -o run --output-format csv -- \
  python3 tools/bench_configs.py --only decbatch --reps 5 > gpurun_out/$O/dec_trace.log 2>&1 || { tail -20 gpurun_out/$O/dec_trace.log; exit 1; }
find gpurun_out/$O/dec_trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/$O/dec_kernel_stats.csv \;
grep -i "brick" gpurun_out/$O/dec_kernel_stats.csv | cut -c1-250
for e in 1024 2048; do
  PROBE_EDGE=$e PROBE_MODES=library PROBE_ITERS=6 timeout -k 10 600 python3 tools/alloc_probe.py > gpurun_out/$O/alloc$e.log 2>&1 || { tail -20 gpurun_out/$O/alloc$e.log; exit 1; }
  tail -2 gpurun_out/$O/alloc$e.log
done
