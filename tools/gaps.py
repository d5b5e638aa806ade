#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace, by (previous, next) pair.
  python tools/gaps.py run_kernel_trace.csv [N]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
gaps = collections.defaultdict(list)
busy = 0
for p, r in zip(rows, rows[1:]):
    gaps[(p['Kernel_Name'][:22], r['Kernel_Name'][:22])].append(int(r['Start_Timestamp']) - int(p['End_Timestamp']))
for r in rows:
    busy += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
span = int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])
print(f"span {span/1e6:.1f} ms, kernels busy {busy/1e6:.1f} ms")
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    v.sort()
    print(f"{k[0]:22s} -> {k[1]:22s} {len(v):6d}  sum {sum(v)/1e6:8.2f} ms  median {v[len(v)//2]/1e3:7.1f} us  p90 {v[int(len(v)*.9)]/1e3:7.1f} us")

# per colouring (k_init ... k_finalize): wall span vs kernel busy time
cur = None
for r in rows:
    nm = r['Kernel_Name']
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if nm.startswith('k_init'):
        cur = [s, 0, 0]
    if cur is not None:
        cur[1] = e
        cur[2] += e - s
    if nm.startswith('k_finalize') and cur is not None:
        print(f"colouring: span {(cur[1]-cur[0])/1e6:7.2f} ms  busy {cur[2]/1e6:7.2f} ms  idle {(cur[1]-cur[0]-cur[2])/1e6:6.2f} ms")
        cur = None
