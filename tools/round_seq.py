#!/usr/bin/env python3
"""Per-round kernel sequence of the last full colouring in a rocprofv3 kernel trace, and the
time per kernel position (sweep k = k-th full-grid JP sweep of its round):
  python tools/round_seq.py run_kernel_trace.csv [round ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_init")]
seq = rows[inits[-2]:inits[-1]]
rounds, cur = [], []
for r in seq:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if n.startswith("k_resolve") and cur:
        rounds.append(cur)
        cur = []
    cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rounds.append(cur)
print(len(rounds), "rounds; span", (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e6, "ms")
for i in [int(x) for x in sys.argv[2:]] or [50, 200, 400, 600, 800]:
    R = rounds[i]
    t0 = R[0][1]
    print(i, f"span {(R[-1][2] - t0) / 1000:.0f}us |", " ".join(f"{n[2:12]}:{(b - a) / 1000:.1f}" for n, a, b in R))
agg, cnt = collections.Counter(), collections.Counter()
busy = 0.0
for R in rounds:
    k = 0
    for n, a, b in R:
        d = (b - a) / 1000
        busy += d
        key = n
        if n == "k_sweep":
            k += 1
            key = f"sweep{k}"
        agg[key] += d
        cnt[key] += 1
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:16]:
    print(f"{k:22s} {v / 1000:7.2f} ms  n={cnt[k]:5d}  avg={v / cnt[k]:6.1f} us")
print("kernel time", busy / 1000, "ms")
