#!/usr/bin/env python3
"""Summarise rocprofv3 output of tools/gpu_profile.sh into per-kernel JSON.

  python tools/pmc_summary.py gpurun_out/<tag> > profiles/<round>/pmc_summary.json

Per kernel name: launches, average duration (kernel trace), and FETCH_SIZE / WRITE_SIZE
per launch from the two separate --pmc passes.  Units: rocprofv3 reports both counters in
KiB; the bytes are given as counted (x1024) and calibrated.

Calibration (round 5, tools/ubench/gather_bytes.hip, profiles/calib/gather_bytes.json):
  * streaming reads, 16 B and 4 B per lane: FETCH_SIZE = 1/2 of the bytes read (as
    MI355X_MICROARCH.md states for 16 B);
  * random 1-B and 4-B gathers past the caches: FETCH_SIZE = 64 B per gather, at a measured
    ceiling of 49.7 G gathers/s -- x2 (the 128-B line the L2 requests) is 6.36 TB/s, the
    HBM's achievable rate, so x2 is the physical reading there too;
  * streaming stores: WRITE_SIZE exact; random 1-B / 4-B stores and 32-bit atomics:
    WRITE_SIZE = 32 B per store (the write granule), counted as moved.
So the calibrated HBM bytes of a kernel are 2 x FETCH_SIZE + WRITE_SIZE.
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", counter) != counter:
            continue
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    return {k: (c, v) for k, (c, v) in agg.items()}


def totals(d, tag):
    f = per_kernel(os.path.join(d, f"pmc_fetch{tag}", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(d, f"pmc_write{tag}", "run_counter_collection.csv"), "WRITE_SIZE")
    return sum(v for _, v in f.values()) * 1024, sum(v for _, v in w.values()) * 1024


def main(d, steps=None):
    stats = {}
    p = os.path.join(d, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(p)):
        stats[r["Name"]] = {"launches": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                            "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])}
    tag = "3" if os.path.isdir(os.path.join(d, "pmc_fetch3")) else ""
    fetch = per_kernel(os.path.join(d, f"pmc_fetch{tag}", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, f"pmc_write{tag}", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["total_ms"]):
        e = dict(s)
        if k in fetch:
            c, v = fetch[k]
            e["fetch_bytes_per_launch"] = v * 1024 / c
            e["fetch_bytes_per_launch_x2_upper"] = 2 * v * 1024 / c
        if k in write:
            c, v = write[k]
            e["write_bytes_per_launch"] = v * 1024 / c
        if "fetch_bytes_per_launch" in e and "write_bytes_per_launch" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"]
            # calibrated: FETCH_SIZE counts half of every read line (streams and gathers alike)
            e["hbm_bytes_per_launch_calibrated"] = 2 * e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"]
        out[k] = e
    if tag == "3" and os.path.isdir(os.path.join(d, "pmc_fetch1")):
        f3, w3 = totals(d, "3")
        f1, w1 = totals(d, "1")
        fb, wb = (f3 - f1) / 2, (w3 - w1) / 2
        out["_step"] = {"steps": 1, "bytes": fb + wb, "fetch_bytes": fb, "write_bytes": wb,
                        "bytes_calibrated": 2 * fb + wb,
                        "note": "FETCH_SIZE + WRITE_SIZE of every kernel, (run at 3 timed steps - run at 1) / 2: "
                                "one step, as counted (KiB x 1024)"}
    # the build the counters describe: bench.py uses a summary only for the same libgcolor.so
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402
    out["_build"] = bench.lib_sha16()
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
