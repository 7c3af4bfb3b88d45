#!/bin/bash
# rocprofv3 kernel trace of one tools/bench_configs.py group: bash scripts/gpu_trace_config.sh <group>
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
G=${1:-config3}
OUT=gpurun_out/trace_$G
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/bench_configs.py --only $G --reps 3 > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
grep '^{' $OUT/log.txt
python3 - "$OUT" <<'PY'
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        print(f'{r["Name"][:110]:110s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:10.1f}')
PY
