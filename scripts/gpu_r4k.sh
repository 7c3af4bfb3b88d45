#!/bin/bash
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4k}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest tests/test_decompose.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -2 gpurun_out/$O/pytest.log
timeout -k 10 600 python3 tools/bench_configs.py --only decpipe --reps 10 > gpurun_out/$O/decpipe.bench.log 2>&1 || { tail -20 gpurun_out/$O/decpipe.bench.log; exit 1; }
grep "^{" gpurun_out/$O/decpipe.bench.log | cut -c1-230
