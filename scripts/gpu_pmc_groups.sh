#!/bin/bash
# bench_configs groups: event timings, then FETCH_SIZE / WRITE_SIZE / SQ passes per dispatch
# (scripts/pmc_dispatch.py).  Output: gpurun_out/$1/.   bash scripts/gpu_pmc_groups.sh <out> <group>...
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for g in "$@"; do
  timeout -k 10 300 python3 tools/bench_configs.py --only $g --reps 10 > $O/$g.bench.log 2>&1 || { tail -20 $O/$g.bench.log; exit 1; }
  grep '^{' $O/$g.bench.log
  B="python3 tools/bench_configs.py --only $g --reps 2"
  timeout -k 10 200 python3 tools/bench_configs.py --only $g --reps 2 > $O/$g.pmc_cases.log 2>&1 || exit 1
  i=0
  PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_ANY")
  [ -n "${PMC_EXTRA:-}" ] && PASSES+=("$PMC_EXTRA")   # one more pass (<= 8 SQ counters)
  # PMC_PASSES="a b;c d": replaces the passes (each within the per-block limits)
  [ -n "${PMC_PASSES:-}" ] && IFS=';' read -r -a PASSES <<< "$PMC_PASSES"
  for pass in "${PASSES[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/$g/p$i -o run --output-format csv -- $B > $O/$g.p$i.log 2>&1 || { tail -20 $O/$g.p$i.log; exit 1; }
    i=$((i+1))
  done
  python3 scripts/pmc_dispatch.py $O/$g $O/$g.pmc_cases.log 3 ${PMC_KERNEL:-} > $O/$g.pmc.jsonl && cat $O/$g.pmc.jsonl
done
