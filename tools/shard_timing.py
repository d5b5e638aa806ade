#!/usr/bin/env python3
"""Rehearse the sharded engine with P shards on ONE GPU (threads, no network): how much
the seam exchanges and per-phase host syncs cost next to the single-GPU engine.

  python tools/shard_timing.py WORKLOAD [parts...]     WORKLOAD: rmat24 | mesh256 | uniform10M | rmat20

Shard views resolve hubs by row scans (no hub JP: its pushed state is not exchanged) but
propose them from hub bitmaps, so the engine with GC_HUB_T=off (no bitmaps either) is only
an approximate single-GPU reference for the seam overhead; the hub engine's time is
printed beside it.  The P shards share one device and one stream, so
their kernels run one after another: the P-shard time is the sum of the shards' kernels
plus the seams, and `seams` below is that time minus the P-way split of the engine's
kernels (an estimate of what the exchange protocol costs per colouring)."""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
import torch  # noqa: E402

from gcolor_amd import shard as sh  # noqa: E402
from gcolor_amd.engine import DeviceGraph, uniform_csr  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "rmat24"
parts_list = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
torch.cuda.set_device(0)
if wl.startswith("rmat"):
    dg = DeviceGraph.rmat(int(wl[4:]), 16, seed=1)
elif wl.startswith("mesh"):
    d = int(wl[4:])
    dg = DeviceGraph.mesh(d, d, d)
else:
    rp, col = uniform_csr(10_000_000 if wl == "uniform10M" else 1_000_000, 16, 42)
    dg = DeviceGraph.from_csr(rp, col, symmetric=True)


def engine_ms(env=None):
    if env:
        os.environ.update(env)
    dg.color("A", want_rounds=False)
    t0 = time.perf_counter()
    for _ in range(3):
        r = dg.color("A", want_rounds=False)
    dt = (time.perf_counter() - t0) / 3 * 1e3
    for k in (env or {}):
        del os.environ[k]
    return dt, r


hub_ms, one = engine_ms()
scan_ms, _ = engine_ms({"GC_HUB_T": "off"})
out = {"workload": wl, "engine_ms": round(hub_ms, 1), "engine_rowscan_ms": round(scan_ms, 1),
       "rounds": one.rounds, "shards": {}}
print(json.dumps(out), flush=True)


def run_parts(shards, **kw):
    hub = sh.ThreadHub(len(shards))
    res, err = [None] * len(shards), []

    def go(i):
        try:
            res[i] = sh.shard_color(shards[i], sh.ThreadTransport(hub, i), want_colors=False, **kw)
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
    return res


rp_d, _ = dg.export(col=False)
for p in parts_list:
    shards = [sh.HipShard(dg, lo, hi) for lo, hi in sh.balanced_ranges(rp_d, p)]
    torch.cuda.synchronize()
    run_parts(shards)
    t0 = time.perf_counter()
    res = run_parts(shards)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    colors, _ = shards[0].colors(False)
    ok = bool((colors == one.colors).all()) if one.colors is not None else None
    seams = res[0].exchanges
    e = {"ms": round(dt, 1), "exchanges": seams, "dense": res[0].dense_exchanges,
         "seam_overhead_ms_est": round(dt - scan_ms, 1), "per_exchange_us": round((dt - scan_ms) * 1e3 / max(seams, 1), 1),
         "identical": ok}
    out["shards"][p] = e
    print(p, json.dumps(e), flush=True)
    for s in shards:
        s.close()
print(json.dumps(out))
