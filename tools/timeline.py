#!/usr/bin/env python3
"""Print the kernel timeline of one colouring (between two k_init launches) from a
rocprofv3 kernel trace: python tools/timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv [k]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
only_busy = len(sys.argv) > 3
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "k_init"]
s, e = idx[-k], idx[-k + 1]
t0 = int(rows[s]["Start_Timestamp"])
prev = None
busy = 0.0
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev) / 1000 if prev else 0.0
    d = (en - st) / 1000
    busy += d
    if not only_busy or d > 10:
        print(f'{r["Kernel_Name"][:22]:22s} dur={d:8.1f} gap={gap:6.1f} t={(st - t0) / 1000:8.1f}')
    prev = en
print(f"launches={e - s} busy_us={busy:.1f} span_us={(prev - t0) / 1000:.1f}")
