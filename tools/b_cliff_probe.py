#!/usr/bin/env python3
"""GPU box: variant B's fold at 7 workgroups per CU (the cliff: every workgroup resident,
profiles/r05/e) under give-up budgets of 20 / 200 ms -- does a launch that gave up at 20 ms
finish when allowed longer (slow progress), or give up again (a stall)?  Device ms and
give-ups per colouring of R-MAT-20."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = f"""
import sys, numpy as np
sys.path[:0] = [{os.path.join(REPO, 'distributed-graph-coloring-with-pyspark_amd')!r}]
from gcolor_amd.engine import DeviceGraph
with DeviceGraph.rmat(20, 16, seed=5) as dg:
    r = [dg.color('B') for _ in range(2)]
    print('ms', [round(x.device_ms, 1) for x in r], 'aborts', [x.async_aborts for x in r], flush=True)
"""
for bpc, budget in (("4", "20000"), ("7", "20000"), ("7", "200000"), ("6", "20000")):
    env = dict(os.environ, GC_B_ASYNC_BPC=bpc, GC_ASYNC_BUDGET_US=budget)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"bpc {bpc} budget {budget} us: {p.stdout.strip()}", flush=True)
    if p.returncode:
        print(p.stderr[-2000:])
        sys.exit(p.returncode)
