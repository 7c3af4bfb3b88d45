#!/bin/bash
# Round-end evidence, every step under its own limit, stopping at the first failure.
#   bash scripts/gpu_final.sh <out> 1   smoke -> GPU tests -> default bench -> rocprofv3 kernel stats
#                                       of the bench -> FETCH_SIZE / WRITE_SIZE / request-size PMC
#                                       passes (separate runs) -> parse
#   bash scripts/gpu_final.sh <out> 2   kernel stats of every tools/bench_configs.py group (under
#                                       rocprofv3 kernel tracing) and the grid-size sweep
# Output: gpurun_out/<out>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
PART=${2:-1}
mkdir -p $O
step() {  # name, limit, command...
    local name=$1 limit=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "$O/$name.log" | cut -c1-400
    return $rc
}
if [ "$PART" = 1 ]; then
    B="python3 bench.py --no-cpu-baseline --no-copy-peak --no-config4"
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
    step bench 300 python bench.py || exit 1
    step prof_trace 300 rocprofv3 --kernel-trace --stats -d $O/prof/trace -o run --output-format csv -- $B || exit 1
    step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof/fetch -o run --output-format csv -- $B || exit 1
    step prof_write 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof/write -o run --output-format csv -- $B || exit 1
    step prof_req 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $O/prof/req -o run --output-format csv -- $B || exit 1
    python3 scripts/parse_pmc.py $O/prof 1024 > $O/pmc_summary.json || exit 1
else
    step configs 900 rocprofv3 --kernel-trace --stats -d $O/configs -o run --output-format csv -- python3 tools/bench_configs.py --reps 5 || exit 1
    grep -c '^{' $O/configs.log
    step sizes 300 python3 tools/bench_sizes.py || exit 1
fi
echo done
