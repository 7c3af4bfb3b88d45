#!/bin/bash
# Bench evidence for the round: the default bench line, the same command under rocprofv3
# kernel-trace/stats, then FETCH_SIZE and WRITE_SIZE in passes of their own (one counter
# block each, as the MI355X guide prescribes), summarised by scripts/parse_pmc.py.  Every step
# has its own time limit; the script stops at the first failure.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-evidence}
mkdir -p $O
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 2 "$O/$name.log" | cut -c1-300
    return $rc
}
B="python3 bench.py --no-cpu-baseline --no-copy-peak --no-secondary"
step bench 400 python3 bench.py || exit 1
step prof_trace 300 rocprofv3 --kernel-trace --stats -d $O/prof/trace -o run --output-format csv -- $B || exit 1
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof/fetch -o run --output-format csv -- $B || exit 1
step prof_write 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof/write -o run --output-format csv -- $B || exit 1
python3 scripts/parse_pmc.py $O/prof 1024 > $O/pmc_summary.json || exit 1
echo done
