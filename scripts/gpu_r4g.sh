#!/bin/bash
# Round-4: BrickDecompose without the per-call descriptor table on uniform grids: parity + timings.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r4g}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest tests/test_decompose.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -60 gpurun_out/$O/pytest.log; exit 1; }
tail -2 gpurun_out/$O/pytest.log
timeout -k 10 600 python3 tools/bench_configs.py --only decbatch --reps 10 > gpurun_out/$O/decbatch.bench.log 2>&1 || { tail -20 gpurun_out/$O/decbatch.bench.log; exit 1; }
grep "^{" gpurun_out/$O/decbatch.bench.log | cut -c1-220
timeout -k 10 120 python3 tools/dec_timing.py > gpurun_out/$O/dec_timing.log 2>&1 || { tail -20 gpurun_out/$O/dec_timing.log; exit 1; }
cat gpurun_out/$O/dec_timing.log
