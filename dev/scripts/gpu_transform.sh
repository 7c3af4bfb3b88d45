#!/bin/bash
# Transform device-functor parity + kernel stats.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-transform}
mkdir -p $O
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$O/$name.log"
    return $rc
}
step pytest 600 python -u -m pytest tests/test_transform_device.py tests/test_gpu_parity.py -k "transform or functor or alias or checker or bench_entry or whole or rejected or larger or 1024_uint8" -x -v --timeout 120 --timeout-method thread || exit 1
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench_configs.py --only transform --reps 10 || exit 1
echo done
