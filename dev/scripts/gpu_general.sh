#!/bin/bash
# General vector path: its parity tests, then the whole GPU suite, then the general-case
# benchmark under rocprofv3.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-general}
mkdir -p $O
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 4 "$O/$name.log"
    return $rc
}
step general_tests 300 python -u -m pytest tests/test_gpu_general.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step general_bench 200 python tools/bench_configs.py --only general --reps 10 || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench_configs.py --only general --reps 10 || exit 1
echo done
