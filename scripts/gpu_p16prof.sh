#!/bin/bash
set -u
# rocprofv3 kernel trace of the packed-16 histogram over volume sizes (tools/bench_configs.py --only p16size).
cd /root/repo; export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_configs.py --only p16size --reps 5 > $O/p16.log 2>&1 || { tail $O/p16.log; exit 1; }
grep '^{' $O/p16.log | cut -c1-140
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
find $O/prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
echo done
