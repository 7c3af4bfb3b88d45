#!/bin/bash
# Round 5: failed-migration tests first, then the whole GPU suite, then the default bench.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "failed_migration or large_migrations" -x -v --timeout 120 --timeout-method thread > $O/mig.log 2>&1 || { tail -40 $O/mig.log; exit 1; }
tail -3 $O/mig.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
