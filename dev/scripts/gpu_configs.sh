#!/bin/bash
# Every tools/bench_configs.py group under rocprofv3 kernel-trace/stats (one bounded step),
# after the full GPU suite.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-configs}
mkdir -p $O
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 2 "$O/$name.log" | cut -c1-200
    return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
step configs 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench_configs.py --reps 5 || exit 1
echo done
