#!/usr/bin/env python3
"""Top kernels of a rocprofv3 run_kernel_stats.csv: calls, average and total time.
  python tools/kstats.py STATS_CSV [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for r in rows[:n]:
    print(f"{r['Name'][:28]:28s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} us {int(r['TotalDurationNs'])/1e6:9.2f} ms")
