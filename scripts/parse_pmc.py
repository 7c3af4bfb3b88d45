"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts exactly half of the bytes of
a wide coalesced streaming read (128-B requests tallied at 64 B), so it is doubled here;
WRITE_SIZE reads exact bytes for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern, counter):
    vals = defaultdict(list)
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                vals[name].append(float(row["Counter_Value"]))
    return vals


def short(name):
    for key, label in (("ArithF<0, 5, 5, 5", "SumRange(UInt16)"), ("IntArithU16F<0>", "SumRange(UInt16)"), ("resamplePlaneKernel", "Resample(replicate)"), ("resampleRowKernel", "Resample(replicate)"), ("resampleRepKernel", "Resample(replicate)"),
                       ("synthKernel", "Synthesize")):
        if key in name:
            return label
    return name[:80]


def main():
    root = sys.argv[1]
    dst_edge = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    fetch = load(os.path.join(root, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(root, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    out = {"note": "bytes per launch; FETCH_SIZE doubled per the gfx950 correction",
           "bench_dst_edge": dst_edge, "kernels": {}}
    for name in set(fetch) | set(write):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out["kernels"][short(name)] = {
            "launches": max(len(f), len(w)),
            "read_bytes": fb, "write_bytes": wb,
            "total_bytes": (fb or 0) + (wb or 0),
        }
    # calibrated reads (when a request-size pass exists): 32 / 64 / 128-B L2 -> fabric requests
    req = {c: load(os.path.join(root, "req", "**", "*counter_collection.csv"), c)
           for c in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")}
    for name in req["TCC_EA0_RDREQ_128B_sum"]:
        k = out["kernels"].get(short(name))
        if k is None:
            continue
        mean = lambda c: sum(req[c].get(name, [0.0])) / max(1, len(req[c].get(name, [])))  # noqa: E731
        k["read_bytes_by_request_size"] = (32 * mean("TCC_EA0_RDREQ_32B_sum") + 64 * mean("TCC_EA0_RDREQ_64B_sum") +
                                           128 * mean("TCC_EA0_RDREQ_128B_sum"))
    s = out["kernels"].get("SumRange(UInt16)")
    if s:
        out["SumRange_bytes_per_launch"] = s["total_bytes"]
    r = out["kernels"].get("Resample(replicate)")
    if r:
        out["Resample_bytes_per_launch"] = r["total_bytes"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
