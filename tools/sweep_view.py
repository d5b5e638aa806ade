#!/usr/bin/env python3
"""Where the JP sweeps of the last colouring in a rocprofv3 kernel trace spend their time:
python tools/sweep_view.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
s = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_init"][-1]
rounds, cur = [], []
for r in rows[s:]:
    n, d = r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    cur.append((n, d))
    if n == "k_close":
        rounds.append(cur)
        cur = []
mx = small = mid = big = 0.0
nsm = nmid = 0
for R in rounds:
    sw = [d for n, d in R if n == "k_sweep"]
    if not sw:
        continue
    m = max(sw)
    mx += m
    rest = list(sw)
    rest.remove(m)
    for x in rest:
        if x < 12:
            small += x
            nsm += 1
        elif x < 50:
            mid += x
            nmid += 1
        else:
            big += x
tot = collections.Counter()
cnt = collections.Counter()
for r in rows[s:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[r["Kernel_Name"]] += d
    cnt[r["Kernel_Name"]] += 1
wall = (int(rows[-1]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e6
print(f"rounds {len(rounds)}  wall {wall:.1f} ms  kernels {sum(tot.values()):.1f} ms")
print(f"sweeps: max-per-round {mx / 1000:.1f} ms, other >50us {big / 1000:.1f}, 12-50us {mid / 1000:.1f} ({nmid}), "
      f"<12us {small / 1000:.1f} ({nsm})")
for k, v in tot.most_common(10):
    print(f"  {k:22s} {v:8.1f} ms  {cnt[k]:6d}")
