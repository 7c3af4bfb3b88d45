#!/bin/bash
# Round-4: Float32 / UInt8 general-path counters (32-bit path at 4 GiB), migrate rates, arena
# steadiness at 2048^3 (5 reallocations), size sweep.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4e}
mkdir -p gpurun_out/$O
bash scripts/gpu_pmc_groups.sh $O f32shift || exit 1
timeout -k 10 300 python3 tools/migrate_bench.py > gpurun_out/$O/migrate.log 2>&1 || { tail -20 gpurun_out/$O/migrate.log; exit 1; }
cat gpurun_out/$O/migrate.log
PROBE_EDGE=2048 PROBE_MODES=library,default PROBE_ITERS=5 timeout -k 10 600 python3 tools/alloc_probe.py > gpurun_out/$O/alloc2048.log 2>&1 || { tail -20 gpurun_out/$O/alloc2048.log; exit 1; }
tail -4 gpurun_out/$O/alloc2048.log
timeout -k 10 300 python3 tools/bench_sizes.py > gpurun_out/$O/sizes.log 2>&1 || { tail -20 gpurun_out/$O/sizes.log; exit 1; }
grep '^{' gpurun_out/$O/sizes.log | cut -c1-300
