#!/bin/bash
# Two ranks of bench.py on one GPU over gloo (the multi-rank bench path rehearsed on a 1-GPU box).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-one-device --dist-backend gloo --dst 256 --config4-edge 512 --no-migrate > $O/reh2.log 2>&1; rc=$?
grep '^{' $O/reh2.log | cut -c1-600; tail -3 $O/reh2.log | cut -c1-300; exit $rc
