#!/bin/bash
# BrickDecompose LDS-write variants: parity, in-process A/B, and LDS stall counters per variant.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-decomp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_decompose.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 tools/bench_configs.py --only decab --reps 10 > $O/decab.log 2>&1 || { tail -20 $O/decab.log; exit 1; }
grep '^{' $O/decab.log
for k in 0; do
  VKT_KNOBS=decompose.aligned_lds=$k timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc$k -o run --output-format csv -- python3 tools/bench_configs.py --only decpmc --reps 2 > $O/pmc$k.log 2>&1 || { tail -20 $O/pmc$k.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
for k in (0, 1, 2):
    tot = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/pmc{k}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "brickCopy" in r["Kernel_Name"]:
                tot[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (d, c), v in tot.items():
        per[c].append(sum(v))
    print("aligned_lds", k, {c: sorted(v)[len(v) // 2] for c, v in sorted(per.items())})
PY
