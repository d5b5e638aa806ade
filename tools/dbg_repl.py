"""Debug helper: sharded colourings with replicated hubs vs one GPU, per configuration."""
import os
import sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "distributed-graph-coloring-with-pyspark_amd"),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
os.environ.setdefault("GC_HUB_T", "8")
from gcolor_amd.engine import DeviceGraph  # noqa: E402
from gcolor_amd import shard as sh  # noqa: E402


def rnd(n, m, seed):
    rng = np.random.default_rng(seed)
    src = np.sort(rng.integers(0, n, m))
    dst = rng.integers(0, n, m)
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


rp, col = rnd(3000, 15000, 0)
with DeviceGraph.from_csr(rp, col) as dg:
    one = dg.color("A")
    print("one  U", list(one.round_U)[:6], "F", list(one.round_F)[:6], "acc", list(one.round_accepted)[:6], flush=True)
    for parts in (1, 2, 3):
        for kw in ({"dense": False}, {"dense": True}):
            r = sh.color_threads(dg, parts, track_rounds=True, **kw)[0]
            ok = np.array_equal(r.colors, one.colors)
            print(parts, kw, ok, "U", r.round_U[:6], "F", r.round_F[:6], "acc", r.round_accepted[:6], flush=True)
            if not ok:
                d = np.nonzero(r.colors != one.colors)[0]
                print("   first diffs", d[:10], "deg", np.diff(rp)[d[:10]], "round one", one.colored_round[d[:10]],
                      "round sh", r.colored_round[d[:10]], flush=True)
