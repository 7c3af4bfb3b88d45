#!/bin/bash
# Multi-row sub-box evidence (UInt8 / Float32): pointwise parity, event timings, FETCH/WRITE and
# SQ passes per dispatch.  Output: gpurun_out/$1/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-subrows}
GRP=${2:-u8sub,f32sub}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_general.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for g in ${GRP//,/ }; do
  timeout -k 10 300 python3 tools/bench_configs.py --only $g --reps 10 > $O/$g.bench.log 2>&1 || { tail -20 $O/$g.bench.log; exit 1; }
  grep '^{' $O/$g.bench.log
  B="python3 tools/bench_configs.py --only $g --reps 2"
  timeout -k 10 200 python3 tools/bench_configs.py --only $g --reps 2 > $O/$g.pmc_cases.log 2>&1 || exit 1
  i=0
  for pass in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
    timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/$g/p$i -o run --output-format csv -- $B > $O/$g.p$i.log 2>&1 || { tail -20 $O/$g.p$i.log; exit 1; }
    i=$((i+1))
  done
  python3 scripts/pmc_dispatch.py $O/$g $O/$g.pmc_cases.log 3 > $O/$g.pmc.jsonl && cat $O/$g.pmc.jsonl
done
