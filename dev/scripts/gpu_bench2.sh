#!/bin/bash
# bench.py: default line, small contract test, 2-rank gloo rehearsal on one device.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-bench2}
mkdir -p $O
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "$O/$name.log"
    return $rc
}
step test_bench 300 python -u -m pytest tests/test_bench.py -x -q --timeout 250 --timeout-method thread || exit 1
step rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --rehearse-one-device --steps 5 --warmup 2 --no-cpu-baseline --dst 512 || exit 1
step bench 400 python bench.py || exit 1
echo done
