"""R-MAT beyond 2^31 adjacency entries (scale 27: ~4.2e9) on one GPU: the engine's
colouring, its validation, and a one-shard sharded colouring against it (the weak-scaling
bench at 8 GPUs colours R-MAT-27; every rank holds the whole CSR)."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
import torch
from gcolor_amd.engine import DeviceGraph
from gcolor_amd import shard as sh
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 27
torch.cuda.set_device(0)
t = time.time()
dg = DeviceGraph.rmat(scale, 16, seed=1)
print(f"R-MAT-{scale}: n {dg.n} nnz {dg.nnz} maxdeg {dg.max_degree} built in {time.time() - t:.1f} s", flush=True)
t = time.time()
r = dg.color("A", want_rounds=False)
print(f"engine: {time.time() - t:.2f} s, device {r.device_ms:.1f} ms, rounds {r.rounds}, colours {r.max_color + 1}, status {r.status}", flush=True)
print("validate", dg.validate(), flush=True)
r2 = dg.color("A", want_rounds=False)
print(f"engine again: device {r2.device_ms:.1f} ms", flush=True)
if len(sys.argv) > 2:
    ops = sh.HipShard(dg, 0, dg.n)
    t = time.time()
    res = sh.shard_color(ops, sh.ThreadTransport(sh.ThreadHub(1), 0))
    print(f"one shard: {time.time() - t:.2f} s, rounds {res.rounds}, identical {np.array_equal(res.colors, r.colors)}", flush=True)
