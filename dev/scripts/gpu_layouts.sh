#!/bin/bash
# Default bench line, then rank 0's slab of the 2/4/8-GPU layouts on one GPU (per-rank time of
# the multi-GPU shapes), then a 2-rank gloo rehearsal of the distributed bench on one device.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log
for M in 2 4 8; do
  timeout -k 10 200 python bench.py --layout-gpus $M --no-cpu-baseline > gpurun_out/bench_layout$M.log 2>&1 || { tail -20 gpurun_out/bench_layout$M.log; exit 1; }
  grep '^{' gpurun_out/bench_layout$M.log
done
bash scripts/gpu_rehearse.sh
