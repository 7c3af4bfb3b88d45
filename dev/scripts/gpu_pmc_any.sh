#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over a command; every pass is its own bounded run.
#   bash scripts/gpu_pmc_any.sh <outdir> "<counters pass 1>" ["<counters pass 2>" ...] -- <cmd...>
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
passes=()
while [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
mkdir -p $OUT
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $p -d $OUT/p$i -o run --output-format csv -- "$@" > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        out[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in out.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   ", c, [round(x) for x in v])
PY
