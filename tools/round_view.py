#!/usr/bin/env python3
"""Per-round kernel view of the last colouring in a rocprofv3 kernel trace:
python tools/round_view.py gpurun_out/<tag>/trace/run_kernel_trace.csv [round ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
s = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_init"][-1]
want = {int(a) for a in sys.argv[2:]}
rounds, cur, rd = [], collections.defaultdict(float), 0
for r in rows[s:]:
    n, d = r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    cur[n] += d
    if rd in want:
        print(rd, n, f"{d:.1f}")
    if n == "k_close":
        rounds.append(cur)
        cur, rd = collections.defaultdict(float), rd + 1
for lo, hi in [(0, 20), (20, 100), (100, 300), (300, 600), (600, 1000), (1000, 10**6)]:
    b = collections.defaultdict(float)
    for x in rounds[lo:hi]:
        for k, v in x.items():
            b[k] += v
    print(lo, hi, {k: round(v / 1000, 1) for k, v in sorted(b.items(), key=lambda x: -x[1])[:6]})
