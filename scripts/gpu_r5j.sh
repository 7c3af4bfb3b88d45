#!/bin/bash
# Round 5: parity (row kernel UInt8/UInt16, memset, decompose), UInt16 row-kernel A/B, decompose
# kernel-only times for aligned_lds 0 vs 3 (rocprofv3 kernel trace + SQ pass), bench.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_memset.py tests/test_decompose.py -x -q --timeout 120 --timeout-method thread > $O/pytest_md.log 2>&1 || { tail -40 $O/pytest_md.log; exit 1; }
tail -2 $O/pytest_md.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_general.py -k "row_kernel or collapsed" -x -q --timeout 120 --timeout-method thread > $O/pytest_row.log 2>&1 || { tail -40 $O/pytest_row.log; exit 1; }
tail -2 $O/pytest_row.log
timeout -k 10 400 python3 tools/bench_configs.py --only u16row --reps 10 > $O/u16row.log 2>&1 || { tail -20 $O/u16row.log; exit 1; }
grep -c '^{' $O/u16row.log
for k in 0 3; do
  VKT_KNOBS=decompose.aligned_lds=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dec$k -o run --output-format csv -- python3 tools/bench_configs.py --only dec16 --reps 10 > $O/dec$k.log 2>&1 || { tail -20 $O/dec$k.log; exit 1; }
  VKT_KNOBS=decompose.aligned_lds=$k timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY -d $O/decpmc$k/p0 -o run --output-format csv -- python3 tools/bench_configs.py --only dec16 --reps 2 > $O/decpmc$k.log 2>&1 || { tail -20 $O/decpmc$k.log; exit 1; }
  python3 scripts/pmc_dispatch.py $O/decpmc$k $O/decpmc$k.log 3 brickCopy > $O/decpmc$k.jsonl && cat $O/decpmc$k.jsonl | cut -c1-300
done
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
