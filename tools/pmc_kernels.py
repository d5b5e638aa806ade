#!/usr/bin/env python3
"""Per-kernel averages of every counter in a rocprofv3 --pmc run_counter_collection.csv.
  python tools/pmc_kernels.py CSV [kernel-substring ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
pats = sys.argv[2:]
for k, cs in sorted(agg.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
    if pats and not any(p in k for p in pats):
        continue
    n = len(next(iter(cs.values())))
    print(k[:40], n, "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
