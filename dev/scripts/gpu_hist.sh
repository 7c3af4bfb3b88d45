#!/bin/bash
# Histogram mul-shift bins: reduce parity tests, then the reduce bench group under rocprofv3.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/hist
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_reduce.py tests/test_gpu_multirank.py tests/test_slab_reduce_gloo.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench_configs.py --only reduce --reps 5 > $O/bench.log 2>&1
rc=$?; grep '^{' $O/bench.log > $O/bench.jsonl; cat $O/bench.jsonl; exit $rc
