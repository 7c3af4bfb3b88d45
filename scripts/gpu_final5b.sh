#!/bin/bash
# Round-5 evidence, part 2: kernel stats of every tools/bench_configs.py group (under
# rocprofv3 kernel tracing) and the grid-size sweep.  Output: gpurun_out/final5/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/final5
mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/configs -o run --output-format csv -- python3 tools/bench_configs.py --reps 5 > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
grep -c '^{' $O/configs.log
timeout -k 10 300 python3 tools/bench_sizes.py > $O/sizes.log 2>&1 || { tail -20 $O/sizes.log; exit 1; }
tail -4 $O/sizes.log
