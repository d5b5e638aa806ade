#!/usr/bin/env python3
"""Debug aid: k_sweep_async's give-up path (GC_ASYNC_BUDGET_US=0) on small graphs, against the
oracle; prints pass / the first divergence per setting.  Usage: tools/dbg_async.py"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))

CHILD = r'''
import os, sys, numpy as np
sys.path[:0] = [os.path.join(R, "tests"), R, os.path.join(R, "distributed-graph-coloring-with-pyspark_amd")]
from test_gpu_parity import _random_directed
from gcolor_amd.engine import DeviceGraph
from oracle import oracle
kind, seed = sys.argv[1], int(sys.argv[2])
if kind == "dir":
    rp, col = _random_directed(2000, 12000, seed)
    sym = False
else:
    from gcolor_amd.generators import reference_csr
    import random
    rp, col = reference_csr(3000, 8, random.Random(seed))
    sym = True
o = oracle.c_color(rp, col, "A")
with DeviceGraph.from_csr(rp, col, symmetric=sym) as dg:
    try:
        g = dg.color("A")
    except Exception as e:
        print("ERROR", e)
        sys.exit(3)
    same = np.array_equal(g.colors, o["colors"])
    U = list(g.round_U); oU = list(o["round_U"])
    first = next((i for i in range(min(len(U), len(oU))) if U[i] != oU[i]), None)
    print("same" if same else "DIFF", "rounds", g.rounds, len(oU), "first_round_diff", first, "aborts", g.async_aborts,
          "sweeps", g.jp_sweeps)
'''


def main():
    settings = [
        {"GC_HUB_T": "off", "GC_ASYNC_BUDGET_US": "0"},
        {"GC_HUB_T": "0", "GC_ASYNC_BUDGET_US": "0"},
        {"GC_HUB_T": "2", "GC_ASYNC_BUDGET_US": "0"},
        {"GC_HUB_T": "2", "GC_ASYNC_BUDGET_US": "3"},
        {"GC_HUB_T": "2"},
    ]
    for st in settings:
        for kind in ("dir", "gen"):
            for seed in range(3):
                env = dict(os.environ, **st)
                p = subprocess.run([sys.executable, "-c", "R=%r\n" % REPO + CHILD, kind, str(seed)], env=env,
                                   capture_output=True, text=True, timeout=120)
                out = (p.stdout.strip().splitlines() or [""])[-1]
                print(st, kind, seed, "rc", p.returncode, out, flush=True)
                if p.returncode not in (0, 3):
                    print(p.stderr[-2000:])
    # one failing case with the control-block dump
    env = dict(os.environ, GC_HUB_T="2", GC_ASYNC_BUDGET_US="0", GC_DEBUG="1")
    p = subprocess.run([sys.executable, "-c", "R=%r\n" % REPO + CHILD, "dir", "1"], env=env, capture_output=True,
                       text=True, timeout=120)
    lines = p.stderr.splitlines()
    print("\n".join(lines[:60]))
    print("...")
    print("\n".join(lines[-40:]))


if __name__ == "__main__":
    main()
