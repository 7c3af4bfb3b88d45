#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: 2 ranks, both on device 0, gloo for the
# barrier / max-over-ranks.  (The driver runs the real N-GPU bench with RCCL.)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --rehearse-one-device --dst 512 \
    > gpurun_out/rehearse.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearse.log || tail -30 gpurun_out/rehearse.log; exit $rc
