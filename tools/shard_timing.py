#!/usr/bin/env python3
"""Time the sharded engine with P shards on ONE GPU (threads, no network): how much the
seam exchanges and per-phase syncs cost next to the single-GPU engine.
python tools/shard_timing.py [n] [parts...]"""
import collections
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
import torch  # noqa: E402

from gcolor_amd import shard as sh  # noqa: E402
from gcolor_amd.engine import DeviceGraph, uniform_csr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
parts_list = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
torch.cuda.set_device(0)
rp, col = uniform_csr(n, 16, 42)
dg = DeviceGraph.from_csr(rp, col, symmetric=True)
dg.color("A")
t0 = time.perf_counter()
for _ in range(3):
    one = dg.color("A", want_rounds=False)
print(f"single engine: {(time.perf_counter() - t0) / 3 * 1e3:.1f} ms", flush=True)


def run_parts(shards, **kw):
    hub = sh.ThreadHub(len(shards))
    out, err = [None] * len(shards), []

    def go(i):
        try:
            out[i] = sh.shard_color(shards[i], sh.ThreadTransport(hub, i), **kw)
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            hub.barrier.abort()
    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(shards))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return out


rp_d, _ = dg.export()
for p in parts_list:
    t0 = time.perf_counter()
    shards = [sh.HipShard(dg, lo, hi) for lo, hi in sh.balanced_ranges(rp_d, p)]
    torch.cuda.synchronize()
    print(f"{p} shards: create {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    for kw in ({}, {"dense": False}, {"local_sweeps": 1}):
        run_parts(shards, **kw)
        t0 = time.perf_counter()
        for _ in range(2):
            res = run_parts(shards, **kw)
        dt = (time.perf_counter() - t0) / 2
        ok = (res[0].colors == one.colors).all()
        print(f"  {kw or 'default'}: {dt * 1e3:.1f} ms  exchanges={res[0].exchanges} "
              f"dense={res[0].dense_exchanges} identical={ok}", flush=True)
    for s in shards:
        s.close()

# per-phase wall time of one shard (1 part) -------------------------------------------
acc = collections.defaultdict(float)


def timed(obj, name):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        out = f(*a, **k)
        torch.cuda.synchronize()
        acc[name] += time.perf_counter() - t
        return out
    setattr(obj, name, g)


ops = sh.HipShard(dg, 0, dg.n)
for name in ("begin", "propose", "apply", "sweep", "finish", "reseed", "colors", "get_slice", "put_slices"):
    timed(ops, name)
hub = sh.ThreadHub(1)
tr = sh.ThreadTransport(hub, 0)
for name in ("gather_stats", "gather_deltas", "gather_slices"):
    timed(tr, name)
sh.shard_color(ops, tr)
acc.clear()
t0 = time.perf_counter()
sh.shard_color(ops, tr)
print(f"1 shard total {(time.perf_counter() - t0) * 1e3:.1f} ms; per phase (ms):",
      {k: round(v * 1e3, 1) for k, v in acc.items()})
