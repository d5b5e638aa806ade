#!/usr/bin/env python3
"""Two colourings of uniform n (default 10M) with P vertex-range shards on one GPU
(threads), for rocprofv3 --kernel-trace --stats: GPU time of the sharded path per kernel.
python tools/shard_prof.py [n] [P]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
import torch  # noqa: E402

from gcolor_amd import shard as sh  # noqa: E402
from gcolor_amd.engine import DeviceGraph, uniform_csr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 2
torch.cuda.set_device(0)
rp, col = uniform_csr(n, 16, 42)
dg = DeviceGraph.from_csr(rp, col, symmetric=True)
rp_d, _ = dg.export()
shards = [sh.HipShard(dg, lo, hi) for lo, hi in sh.balanced_ranges(rp_d, P)]
import threading  # noqa: E402


def run():
    hub = sh.ThreadHub(P)
    out = [None] * P
    ts = [threading.Thread(target=lambda i=i: out.__setitem__(i, sh.shard_color(shards[i], sh.ThreadTransport(hub, i))))
          for i in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


run()
t0 = time.perf_counter()
res = run()
print(f"P={P}: {(time.perf_counter() - t0) * 1e3:.1f} ms, exchanges {res[0].exchanges}")
for s in shards:
    s.close()
