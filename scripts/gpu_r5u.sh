#!/bin/bash
# Round 5: fixed per-call cost of aggregates / histogram -- wall times, then the same run under
# a kernel + memory-copy trace (kernels per call and the gaps between them).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 200 python3 tools/agg_fixed.py 200 > $O/plain.log 2>&1 || { tail -20 $O/plain.log; exit 1; }
cat $O/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 tools/agg_fixed.py 50 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
ls $O/trace
