#!/usr/bin/env python3
"""Where variant B's colouring time goes, round by round (csrc/gc_variant_b.hip).

  run:      python tools/b_round_cost.py run WORKLOAD OUT.json [COLOURINGS]
            colours the workload's graph with variant B COLOURINGS times (default 2) and writes
            the per-round records (uncoloured U, winners, fold passes); meant to be run under
            `rocprofv3 --kernel-trace -d DIR -- python3 tools/b_round_cost.py run ...`.
  analyze:  python tools/b_round_cost.py analyze KERNEL_TRACE.csv OUT.json
            splits the LAST colouring of the trace at its k_b_reset launches and reports, per
            class of rounds (by U): rounds, fold passes, the first admission pass (every
            proposer), the later admission passes, the eviction passes, and the rest.
"""
import collections
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = [(0, 1024), (1024, 16384), (16384, 262144), (262144, 1 << 62)]


def run(wl, out, colourings):
    sys.path[:0] = [REPO, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")]
    import torch
    import bench
    torch.cuda.set_device(0)
    dg, _ = bench.build_graph(bench.WORKLOADS[wl])
    res = None
    for _ in range(max(colourings, 1)):
        res = dg.color("B")
    with open(out, "w") as f:
        json.dump({"workload": wl, "U": [int(x) for x in res.round_U], "accepted": [int(x) for x in res.round_accepted],
                   "device_ms": res.device_ms, "sweeps": int(res.jp_sweeps)}, f)
    print(f"{wl}: {res.rounds} rounds, device {res.device_ms:.1f} ms, fold passes {res.jp_sweeps} -> {out}")


def analyze(trace, rec_path):
    rec = json.load(open(rec_path))
    U = rec["U"]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].split("<")[0] for r in rows]
    inits = [i for i, nm in enumerate(names) if nm == "k_init"]
    if not inits:
        sys.exit("no colouring in the trace")
    seq = list(zip(names, rows))[inits[-1]:]
    rounds, cur = [], None
    for nm, r in seq:
        if nm.startswith("k_finalize"):
            break
        if nm == "k_b_reset":
            cur = []
            rounds.append(cur)
        if cur is not None:
            cur.append((nm, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"{len(rounds)} rounds in the last colouring (records: {len(U)})")
    agg = collections.OrderedDict((c, collections.Counter()) for c in CLASSES)
    per_round = collections.OrderedDict((c, []) for c in CLASSES)
    async_per_round = []
    for i, rnd in enumerate(rounds):
        # round i's records: U of round i (the last round lists U = 0)
        u = U[i] if i < len(U) else 0
        cls = next(c for c in CLASSES if c[0] <= u < c[1])
        a = agg[cls]
        a["rounds"] += 1
        a["U"] += u
        first = True
        wall = (rnd[-1][2] - rnd[0][1]) / 1e3
        a["wall_us"] += wall
        for nm, t0, t1 in rnd:
            d = (t1 - t0) / 1e3
            a["busy_us"] += d
            if nm == "k_b_adm":
                a["passes"] += 1
                if first:
                    a["adm_first_us"] += d
                    first = False
                else:
                    a["adm_rest_us"] += d
            elif nm == "k_b_ev":
                a["ev_us"] += d
            elif nm == "k_b_async":  # the asynchronous fold (hub graphs): the round's passes in one launch
                a["async_us"] += d
                a["async_n"] += 1
                async_per_round.append((i, u, d))
            else:
                a["other_us"] += d
                a["other:" + nm] += d
        per_round[cls].append(wall)
    hdr = f"{'U class':>16} {'rounds':>6} {'sumU':>10} {'passes':>7} {'wall ms':>8} {'adm1 ms':>8} {'adm+ ms':>8} " \
          f"{'ev ms':>7} {'async ms':>8} {'rest ms':>8} {'med round us':>12}"
    print(hdr)
    for c, a in agg.items():
        if not a["rounds"]:
            continue
        lab = f"[{c[0]}, {c[1] if c[1] < 1 << 40 else 'inf'})"
        print(f"{lab:>16} {a['rounds']:>6} {a['U']:>10} {a['passes']:>7} {a['wall_us'] / 1e3:>8.1f} "
              f"{a['adm_first_us'] / 1e3:>8.1f} {a['adm_rest_us'] / 1e3:>8.1f} {a['ev_us'] / 1e3:>7.1f} "
              f"{a['async_us'] / 1e3:>8.1f} {a['other_us'] / 1e3:>8.1f} {statistics.median(per_round[c]):>12.1f}")
        top = sorted(((k[6:], v) for k, v in a.items() if k.startswith("other:")), key=lambda kv: -kv[1])[:5]
        print(" " * 18 + "rest: " + ", ".join(f"{k} {v / 1e3:.1f}" for k, v in top))
    tw = sum(a["wall_us"] for a in agg.values())
    tb = sum(a["busy_us"] for a in agg.values())
    print(f"rounds' wall {tw / 1e3:.1f} ms, kernels busy {tb / 1e3:.1f} ms, idle {(tw - tb) / 1e3:.1f} ms")
    if async_per_round:
        print("k_b_async per round (round, U, us): first 16 and every 25th")
        sel = async_per_round[:16] + async_per_round[16::25]
        print("  " + "  ".join(f"{i}:{u}:{d:.0f}" for i, u, d in sel))
        ds = sorted(d for _, _, d in async_per_round)
        q = lambda f: ds[min(len(ds) - 1, int(f * len(ds)))]
        print(f"  k_b_async us: p10 {q(0.1):.0f} p50 {q(0.5):.0f} p90 {q(0.9):.0f} max {ds[-1]:.0f}; "
              f"us per U item (U >= 1e4): {statistics.median([d / u for _, u, d in async_per_round if u >= 1e4] or [0]):.4f}")


if __name__ == "__main__":
    if len(sys.argv) >= 4 and sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    elif len(sys.argv) == 4 and sys.argv[1] == "analyze":
        analyze(sys.argv[2], sys.argv[3])
    else:
        sys.exit(__doc__)
