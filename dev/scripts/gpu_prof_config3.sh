#!/bin/bash
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof3
mkdir -p $OUT
B="python3 tools/bench_configs.py --only config3 --reps 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for cnt, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    v = defaultdict(list)
    for p in glob.glob(f"gpurun_out/prof3/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == cnt:
                v[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
    for k, x in v.items():
        print(cnt, k, "avg KB", sum(x) / len(x), "n", len(x))
PY
grep -h '^{' $OUT/trace.log
cut -d, -f1-4 $OUT/trace/run_kernel_stats.csv | cut -c1-150
