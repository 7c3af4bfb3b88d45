#!/bin/bash
# GPU-box validation run: smoke -> parity tests -> short bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (exit > 1) stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name" | tee -a gpurun_out/steps.log
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -n 5 "gpurun_out/$name.log"
    return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
rc=$?; [ $rc -gt 1 ] && exit $rc
step bench 300 python bench.py --steps 10 --warmup 3 || exit $?
cat gpurun_out/bench.log
export TMPDIR=/tmp
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $?
find gpurun_out/prof -name "*stats*" | head
exit 0
