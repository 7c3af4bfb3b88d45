#!/bin/bash
# Round-6 check: smoke, the whole GPU suite, the default bench.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-check6}; mkdir -p $O
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "$O/$name.log" | cut -c1-400
    return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
step bench 300 python bench.py || exit 1
echo done
