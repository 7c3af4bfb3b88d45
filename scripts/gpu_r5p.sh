#!/bin/bash
# Round 5: general-path kernels parity + A/B of one kernel per span path (group gensplit).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_general.py -k "general_path_kernels" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python3 tools/bench_configs.py --only gensplit --reps 10 > $O/gensplit.log 2>&1 || { tail -20 $O/gensplit.log; exit 1; }
grep -c '^{' $O/gensplit.log
