"""Per-dispatch PMC table from rocprofv3 counter CSVs (one directory per pass), in dispatch
order, joined with the case lines a bench printed.

  python3 scripts/pmc_dispatch.py <dir with p0/ p1/ ...> <bench log with JSON case lines> <launches per case> [kernel]

(kernel: only dispatches whose kernel name contains it -- ops that launch several kernels)

Each case of tools/bench_configs.py runs `reps + 1` launches (one warm-up); a case's value is
the median over its launches.  FETCH_SIZE is doubled (gfx950: a wide coalesced read is
counted at half its bytes, MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact.  Both are reported
in bytes; SQ counters as summed over the dispatch.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    root, log, per = sys.argv[1], sys.argv[2], int(sys.argv[3])
    only = sys.argv[4] if len(sys.argv) > 4 else None   # keep dispatches whose kernel name holds this
    disp = defaultdict(dict)   # (pass, dispatch) -> {counter: value}, kernel
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(p):
            continue
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (os.path.basename(p), int(r["Dispatch_Id"]))
                disp[k]["kernel"] = r["Kernel_Name"]
                disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    passes = sorted({k[0] for k in disp})
    cases = [json.loads(line) for line in open(log) if line.startswith("{")]
    out = []
    for pname in passes:
        ds = [disp[k] for k in sorted(k for k in disp if k[0] == pname)]
        # drop the input synthesis / setup kernels: keep dispatches of the measured ops
        ds = [d for d in ds if "synthKernel" not in d["kernel"] and "elementwise" not in d["kernel"]
              and "__amd_rocclr" not in d["kernel"] and "distribution" not in d["kernel"]
              and "fill" not in d["kernel"].lower()[:40]]
        if only:
            ds = [d for d in ds if only in d["kernel"]]
        for i, c in enumerate(cases):
            chunk = ds[i * per:(i + 1) * per]
            if not chunk:
                break
            if len(out) <= i:
                out.append({"case": c["case"], "ms": c.get("ms"), "kernel": chunk[0]["kernel"][:120]})
            for name in chunk[0]:
                if name == "kernel":
                    continue
                v = statistics.median(d.get(name, 0.0) for d in chunk)
                if name == "FETCH_SIZE":
                    out[i]["read_bytes"] = 2 * 1024 * v
                elif name == "WRITE_SIZE":
                    out[i]["write_bytes"] = 1024 * v
                else:
                    out[i][name] = v
    for o in out:
        # calibrated read bytes: the L2 -> fabric read requests by size (gfx950 counts 32-, 64- and
        # 128-B requests separately; FETCH_SIZE tallies the 128-B ones at 64 B -- the "doubling")
        if all(k in o for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
            o["read_bytes_by_req"] = (32 * o["TCC_EA0_RDREQ_32B_sum"] + 64 * o["TCC_EA0_RDREQ_64B_sum"] +
                                      128 * o["TCC_EA0_RDREQ_128B_sum"])
        if "TCC_EA0_WRREQ_sum" in o and "TCC_EA0_WRREQ_64B_sum" in o:
            o["write_bytes_by_req"] = 32 * (o["TCC_EA0_WRREQ_sum"] - o["TCC_EA0_WRREQ_64B_sum"]) + \
                64 * o["TCC_EA0_WRREQ_64B_sum"]
        print(json.dumps(o))


if __name__ == "__main__":
    main()
