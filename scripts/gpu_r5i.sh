#!/bin/bash
# Round 5: UInt8 row-kernel A/B + parity, memory tests, decompose dump-write A/B + parity, bench.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_general.py -k "row_kernel or collapsed" tests/test_memset.py tests/test_decompose.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 tools/bench_configs.py --only u8row --reps 10 > $O/u8row.log 2>&1 || { tail -20 $O/u8row.log; exit 1; }
grep -c '^{' $O/u8row.log
timeout -k 10 400 python3 tools/bench_configs.py --only decdump --reps 10 > $O/decdump.log 2>&1 || { tail -20 $O/decdump.log; exit 1; }
grep '^{' $O/decdump.log | cut -c1-150
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
