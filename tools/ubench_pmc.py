#!/usr/bin/env python3
"""Join tools/ubench/gather_bytes' timing lines with its rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

  python tools/ubench_pmc.py DIR > DIR/calibration.json

DIR holds timing.txt (the program's stdout) and pmc_fetch/, pmc_write/ (rocprofv3 --pmc runs of
the same program, -o run).  Per kernel: the bytes the kernel's ops name (ops x bytes per op), the
counters per launch (KiB x 1024, as counted), their ratio to the named bytes, per op, and the
rate.  The first launch of each kernel is a warm-up and its counters are dropped (the timing
line averages the others).  The result is the calibration DESIGN.md §4 and bench.py's
`pmc_calibration` apply to the engine's gathers.
"""
import collections
import csv
import json
import os
import sys


def counters(path, name):
    rows = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", name) != name:
            continue
        rows[r["Kernel_Name"].split("(")[0].strip()].append((int(r.get("Dispatch_Id", 0) or 0),
                                                             float(r["Counter_Value"]) * 1024))
    out = {}
    for k, v in rows.items():
        v.sort()
        vals = [b for _, b in v[1:]] or [b for _, b in v]  # drop the warm-up launch
        out[k] = sum(vals) / len(vals)
    return out


def find_csv(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    return os.path.join(d, "missing.csv")


def main(d):
    timing = {}
    for line in open(os.path.join(d, "timing.txt")):
        if line.startswith("#") or not line.strip():
            continue
        k, launches, ops, bpo, us = line.split()
        timing[k] = {"ops": int(ops), "bytes_per_op": int(bpo), "avg_us": float(us)}
    fetch = counters(find_csv(os.path.join(d, "pmc_fetch")), "FETCH_SIZE")
    write = counters(find_csv(os.path.join(d, "pmc_write")), "WRITE_SIZE")
    out = {}
    for k, t in timing.items():
        named = t["ops"] * t["bytes_per_op"]
        e = dict(t, named_bytes=named, named_GBps=round(named / t["avg_us"] / 1e3, 1),
                 ops_per_s=t["ops"] / (t["avg_us"] / 1e6))
        for tag, src in (("fetch", fetch), ("write", write)):
            if k in src:
                b = src[k]
                e[f"{tag}_bytes"] = b
                e[f"{tag}_over_named"] = round(b / named, 4)
                e[f"{tag}_bytes_per_op"] = round(b / t["ops"], 3)
                e[f"{tag}_GBps_as_counted"] = round(b / t["avg_us"] / 1e3, 1)
        out[k] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
