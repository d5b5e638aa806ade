#!/usr/bin/env python3
"""Per-kernel duration quantiles of one colouring in a rocprofv3 kernel trace, split into
the colouring's first, middle and last thirds of rounds (k_close / k_commit mark rounds).
  python tools/round_kernels.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last full colouring: from the last k_init to the k_finalize after it
starts = [i for i, r in enumerate(rows) if r['Kernel_Name'].startswith('k_init')]
i0 = starts[-2] if len(starts) > 1 else starts[-1]
i1 = next(i for i in range(i0, len(rows)) if rows[i]['Kernel_Name'].startswith('k_finalize'))
seq = rows[i0:i1 + 1]
rnd, per = 0, []
for r in seq:
    nm = r['Kernel_Name'].split('(')[0]
    per.append((rnd, nm, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
    if nm.startswith('k_close'):
        rnd += 1
R = max(rnd, 1)
for third in range(3):
    lo, hi = third * R // 3, (third + 1) * R // 3
    agg = collections.defaultdict(list)
    for k, nm, us in per:
        if lo <= k < hi:
            agg[nm].append(us)
    tot = sum(sum(v) for v in agg.values())
    print(f"rounds [{lo},{hi}): {tot / 1e3:.1f} ms")
    for nm, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:9]:
        v.sort()
        print(f"  {nm[:22]:22s} n={len(v):5d} sum={sum(v)/1e3:7.2f} ms  p50={v[len(v)//2]:7.1f} us  p90={v[int(len(v)*.9)]:7.1f} us")
