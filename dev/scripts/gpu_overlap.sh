#!/bin/bash
# Overlapped halo exchange: 2-rank GPU test + the reduce guard, then a 2-rank bench rehearsal
# on one GPU (gloo staging; RCCL needs two GPUs).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/overlap
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py tests/test_reduce.py -m gpu -x -q --timeout 300 --timeout-method thread -k "two_ranks or integer_pass" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --rehearse-one-device --dst 512 \
    > $O/rehearse.log 2>&1
rc=$?; grep '^{' $O/rehearse.log || tail -30 $O/rehearse.log; exit $rc
