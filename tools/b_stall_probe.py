#!/usr/bin/env python3
"""GPU box: variant B's asynchronous fold past 6 workgroups per CU (round 5's cliff), with the
state of the first launch that gave up dumped for tools/b_stall_analyze.py (GC_B_STALL_DUMP).
Needs a build of the fold for more waves per SIMD (GC_LIB_PATH, e.g. -DGC_B_WPE=8
-DGC_B_RES_CAP=512).  Writes OUT/stall_bpc*.*.bin (the graph itself is tests/golden/make_rmat_fixtures.py's
numpy replica, seed 5) and prints device ms, give-ups, the measured residency and whether the
colouring equals the oracle's.
Usage: python tools/b_stall_probe.py OUT [scale] [bpc ...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1]
scale = int(sys.argv[2]) if len(sys.argv) > 2 else 20
bpcs = sys.argv[3:] or ["6", "7", "8"]
os.makedirs(out, exist_ok=True)
code = f"""
import os, sys, numpy as np
sys.path[:0] = [{REPO!r}, {os.path.join(REPO, 'distributed-graph-coloring-with-pyspark_amd')!r}]
from gcolor_amd.engine import DeviceGraph
from oracle import oracle
with DeviceGraph.rmat({scale}, 16, seed=5) as dg:
    r = dg.color('B')
    rp, col = dg.export()
    o = oracle.c_color(rp, col, 'B')
    same = bool(np.array_equal(r.colors, o['colors']))
    print('ms', round(r.device_ms, 1), 'aborts', r.async_aborts, 'rounds', r.rounds, 'equal to oracle', same, flush=True)
"""
for bpc in bpcs:
    env = dict(os.environ, GC_B_ASYNC_BPC=bpc, GC_DEBUG="1",
               GC_B_STALL_DUMP=os.path.join(out, f"stall_bpc{bpc}"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=500)
    print(f"bpc {bpc}: {p.stdout.strip()}", flush=True)
    print("   ", "\n    ".join(l for l in p.stderr.splitlines() if "residency" in l), flush=True)
    if p.returncode:
        print(p.stderr[-3000:])
        sys.exit(p.returncode)
