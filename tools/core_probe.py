#!/usr/bin/env python3
"""GPU box: how many rounds the hub core (csrc/gc_core.hip) decides on R-MAT graphs at several
hub thresholds, and whether each colouring equals the oracle's (small graphs) or the same
graph's colouring with the core off (large ones).
Usage: python tools/core_probe.py [scale:T ...]   (default 12:0 14:64 14:512 16:128 18:512 20:512 24:512)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")]
import numpy as np  # noqa: E402

from gcolor_amd.engine import DeviceGraph  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    cases = sys.argv[1:] or ["12:0", "14:64", "14:512", "16:128", "18:512", "20:512", "24:512"]
    for c in cases:
        scale, t = (int(x) for x in c.split(":"))
        os.environ["GC_HUB_T"] = str(t)
        os.environ["GC_HUB_CORE"] = "1"
        with DeviceGraph.rmat(scale, 16, seed=scale) as dg:
            t0 = time.perf_counter()
            g = dg.color("A")
            dt = time.perf_counter() - t0
            os.environ["GC_HUB_CORE"] = "0"
            t1 = time.perf_counter()
            off = dg.color("A")
            dt_off = time.perf_counter() - t1
            os.environ["GC_HUB_CORE"] = "1"
            same_off = np.array_equal(g.colors, off.colors) and np.array_equal(g.round_U, off.round_U)
            same_oracle = None
            if scale <= 16:
                rp, col = dg.export()
                same_oracle = bool(np.array_equal(g.colors, oracle.c_color(rp, col, "A")["colors"]))
        print(f"R-MAT-{scale} T={t}: rounds {g.rounds}, core rounds {g.core_rounds}, hubs {g.hubs}, aborts "
              f"{g.async_aborts}; core on {g.device_ms:.2f} ms (wall {dt * 1e3:.1f}), off {off.device_ms:.2f} ms "
              f"(wall {dt_off * 1e3:.1f}); equal to core off: {same_off}; equal to oracle: {same_oracle}", flush=True)


if __name__ == "__main__":
    main()
