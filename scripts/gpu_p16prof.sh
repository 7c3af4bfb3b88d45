#!/bin/bash
# rocprofv3 kernel trace and FETCH_SIZE / WRITE_SIZE passes of the packed-16 histogram over volume
# sizes (tools/bench_configs.py --only p16size).  Output: gpurun_out/<out>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-p16prof}; mkdir -p $O
C="python3 tools/bench_configs.py --only p16size --reps 3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $C > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $C > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $C > $O/write.log 2>&1 || { tail $O/write.log; exit 1; }
grep '^{' $O/trace.log | cut -c1-120
echo done
