#!/usr/bin/env python3
"""What a colouring round costs on the GPU, by frontier size.

  run:      python tools/round_cost.py run WORKLOAD OUT.json [COLOURINGS]
            colours the workload's graph (bench.WORKLOADS) COLOURINGS times (default 2) and
            writes the per-round records (frontier size F, undecided U, winners) of the run;
            meant to be run under `rocprofv3 --kernel-trace -d DIR -- python3 tools/round_cost.py
            run ...` (the records do not depend on the run: the colouring is deterministic).
  analyze:  python tools/round_cost.py analyze KERNEL_TRACE.csv OUT.json
            splits the LAST colouring of the trace into rounds (a round ends with its k_close,
            or with its closing k_commit when the round had no k_close) and reports, per
            frontier-size class: rounds, their total wall time, and the median wall time,
            kernel busy time, gap time and per-kernel duration of one round.

The split assumes one round per closing kernel, which holds for variant A's engine: an E1
re-seed round also ends with a k_close (its records carry seeds > 0).
"""
import collections
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = [(0, 1024), (1024, 16384), (16384, 65536), (65536, 1 << 62)]


def run(wl, out, colourings):
    sys.path[:0] = [REPO, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")]
    import torch
    import bench
    torch.cuda.set_device(0)
    dg, _ = bench.build_graph(bench.WORKLOADS[wl])
    res = None
    for _ in range(max(colourings, 1)):
        res = dg.color("A")
    with open(out, "w") as f:
        json.dump({"workload": wl, "F": [int(x) for x in res.round_F], "U": [int(x) for x in res.round_U],
                   "accepted": [int(x) for x in res.round_accepted], "seeds": [int(x) for x in res.round_seeds],
                   "device_ms": res.device_ms}, f)
    print(f"{wl}: {res.rounds} rounds, device {res.device_ms:.1f} ms -> {out}")


def analyze(trace, rec_path):
    rec = json.load(open(rec_path))
    F = rec["F"]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].split("(")[0] in ("k_init", "k_resume_init")]
    if not starts:
        sys.exit("no colouring in the trace")
    seq = rows[starts[-1]:]
    rounds, cur = [], []
    for i, r in enumerate(seq):
        nm = r["Kernel_Name"].split("(")[0]
        if nm.startswith("k_finalize"):
            break
        cur.append((nm, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        nxt = seq[i + 1]["Kernel_Name"].split("(")[0] if i + 1 < len(seq) else ""
        if nm.startswith("k_close") or (nm.startswith("k_commit") and not nm.startswith("k_commit_big")
                                         and not nxt.startswith(("k_commit_big", "k_close", "k_pull"))):
            rounds.append(cur)
            cur = []
    # the INIT commit closes "round -1" (seed), so round r of the records is rounds[r + 1]
    body = rounds[1:] if len(rounds) > len(F) - 1 else rounds
    n = min(len(body), len(F))
    print(f"{rec['workload']}: {len(F)} records, {len(rounds)} closing kernels in the last colouring; "
          f"comparing {n} rounds")
    for lo, hi in CLASSES:
        sel = [body[r] for r in range(n) if lo <= F[r] < hi]
        if not sel:
            continue
        wall = [(R[-1][2] - R[0][1]) / 1e3 for R in sel]
        busy = [sum(e - s for _, s, e in R) / 1e3 for R in sel]
        gaps = [w - b for w, b in zip(wall, busy)]
        per = collections.defaultdict(list)
        for R in sel:
            acc = collections.defaultdict(float)
            for nm, s, e in R:
                acc[nm] += (e - s) / 1e3
            for nm, us in acc.items():
                per[nm].append(us)
        hi_s = "inf" if hi >= 1 << 62 else str(hi)
        print(f"  F in [{lo}, {hi_s}): {len(sel)} rounds, {sum(wall) / 1e3:.1f} ms; per round median: wall "
              f"{statistics.median(wall):.1f} us = busy {statistics.median(busy):.1f} + gaps {statistics.median(gaps):.1f}")
        for nm, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
            print(f"      {nm:22s} {statistics.median(v):8.1f} us median  ({len(v)} rounds, {sum(v) / 1e3:.1f} ms)")


if __name__ == "__main__":
    if len(sys.argv) >= 4 and sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    elif len(sys.argv) == 4 and sys.argv[1] == "analyze":
        analyze(sys.argv[2], sys.argv[3])
    else:
        sys.exit(__doc__)
