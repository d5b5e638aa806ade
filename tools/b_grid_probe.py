#!/usr/bin/env python3
"""GPU box: variant B's asynchronous fold (k_b_async) and variant A's asynchronous JP at
several workgroups per CU on one R-MAT graph: device ms, give-ups (async_aborts), equal
colours; GC_DEBUG=1 prints the measured residency.  Usage: b_grid_probe.py [scale]."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
scale = sys.argv[1] if len(sys.argv) > 1 else "20"
code = f"""
import sys, numpy as np
sys.path[:0] = [{os.path.join(REPO, 'distributed-graph-coloring-with-pyspark_amd')!r}]
from gcolor_amd.engine import DeviceGraph
with DeviceGraph.rmat({scale}, 16, seed=5) as dg:
    for v in ('B', 'A'):
        r = [dg.color(v) for _ in range(3)]
        print(v, 'ms', [round(x.device_ms, 1) for x in r], 'aborts', [x.async_aborts for x in r], 'colours', r[0].max_color + 1,
              'equal', all(np.array_equal(x.colors, r[0].colors) for x in r), flush=True)
"""
for bpc in ("2", "4", "6", "7", "8"):
    env = dict(os.environ, GC_B_ASYNC_BPC=bpc, GC_ASYNC_BPC=bpc, GC_DEBUG_PROBE="1")
    print(f"== {bpc} workgroups per CU requested", flush=True)
    p = subprocess.run([sys.executable, "-c", code], env=dict(env, GC_DEBUG="1"), capture_output=True, text=True,
                       timeout=300)
    print(p.stdout, end="")
    print("\n".join(l for l in p.stderr.splitlines() if "residency" in l), flush=True)
    if p.returncode:
        print(p.stderr[-2000:])
        sys.exit(p.returncode)
