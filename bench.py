#!/usr/bin/env python3
"""Benchmark: edges coloured per second (TEPS) of the MI355X colouring engine.

Workload (default, BASELINE.json configs[1] = C2): uniform random graph with the
reference generator's process (graph.py:30-43), n = 10M vertices, max degree 16,
seed 42, built on the host by the native generator and copied to HBM once.  A step is
one full colouring (coloring.py:73-132 semantics, variant A) from the resident CSR to
a complete valid colouring; value = m / t (m = undirected edges = nnz/2), whole job.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per
GPU, each colouring its own resident replica of the workload (weak scaling,
parallelism "replicas"); barrier + synchronize around the K timed steps, max time over
ranks; value = N * m / t_max.

Extra objects on the JSON line:
  roofline      dominant kernel class (by time) of one instrumented step: SURVEY.md §8d
                algorithmic bytes / its event-timed duration vs 8 TB/s HBM peak
  cpu_baseline  oracle/gcolor_oracle.c (the C restatement, 1 thread) on the same graph,
                rank 0 at N=1 only
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")
sys.path.insert(0, PKG_DIR)

METRIC = "edges colored/sec (TEPS), colors used, % HBM roofline at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0

WORKLOADS = {
    "uniform10M": dict(kind="uniform", n=10_000_000, d=16, seed=42,
                       desc="C2: uniform (graph.py:30-43 process) n=10M, max-degree 16, seed 42"),
    "rmat24": dict(kind="rmat", scale=24, ef=16, seed=1,
                   desc="C3: R-MAT scale 24, edge factor 16, (0.57,0.19,0.19), seed 1, symmetrised"),
    "rmat26": dict(kind="rmat", scale=26, ef=16, seed=1,
                   desc="north star: R-MAT scale 26, edge factor 16, (0.57,0.19,0.19), seed 1"),
    "mesh512": dict(kind="mesh", dims=(512, 512, 512), desc="C4 (1 GPU): 3-D 7-point mesh 512^3"),
    "mesh256": dict(kind="mesh", dims=(256, 256, 256), desc="3-D 7-point mesh 256^3"),
    "uniform1M": dict(kind="uniform", n=1_000_000, d=16, seed=42, desc="uniform n=1M, max-degree 16"),
}


def build_graph(w):
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    if w["kind"] == "uniform":
        rp, col = uniform_csr(w["n"], w["d"], w["seed"])
        return DeviceGraph.from_csr(rp, col, symmetric=True), (rp, col)
    if w["kind"] == "rmat":
        return DeviceGraph.rmat(w["scale"], w["ef"], seed=w["seed"]), None
    return DeviceGraph.mesh(*w["dims"]), None


KERNEL_OF_CLASS = {"propose": "k_propose", "resolve": "k_resolve", "sweep": "k_sweep", "commit": "k_commit"}


def pmc_traffic(kclass, workload):
    """HBM bytes per launch of the dominant kernel from the rocprofv3 --pmc passes of this
    same bench command (tools/gpu_profile.sh -> tools/pmc_summary.py -> profiles/latest).
    FETCH_SIZE + WRITE_SIZE in KiB x 1024, averaged over all launches of the kernel."""
    p = os.path.join(REPO, "profiles", "latest", "pmc_summary.json")
    name = KERNEL_OF_CLASS.get(kclass)
    if workload != "uniform10M" or not name or not os.path.exists(p):
        return None, None
    e = json.load(open(p)).get(name, {})
    if "hbm_bytes_per_launch" not in e:
        return None, None
    return e["hbm_bytes_per_launch"], "profiles/latest/pmc_summary.json (bytes per launch, FETCH_SIZE+WRITE_SIZE)"


def cpu_baseline(w, host_csr, dg):
    """The C restatement (1 thread) on the same graph; TEPS on the host cores."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    if host_csr is None:
        host_csr = dg.export()
    rp, col = host_csr
    t0 = time.perf_counter()
    o = oracle.c_color(rp, col, "A")
    dt = time.perf_counter() - t0
    m = len(col) / 2
    return {"value": m / dt, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"oracle/gcolor_oracle.c on the full {w['desc']} graph ({dt:.1f} s, 1 thread, "
                      f"{platform.processor() or platform.machine()}, {os.cpu_count()} host CPUs visible)",
            "colors": int(o["max_color"]) + 1, "seconds": dt}, o


def run_sharded(args, world, rank, local_rank, dist, torch):
    """N > 1: ONE graph, vertex-range shards over the N ranks (gcolor_amd.shard), round
    deltas all-gathered over RCCL.  Weak scaling: the per-GPU share is the N=1 workload
    (uniform: n = 10M x N; R-MAT: scale + log2 N; mesh: z x N)."""
    import math
    from gcolor_amd import _native
    from gcolor_amd import shard as sh
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    _native.check("gc_set_device", _native.load().gc_set_device(local_rank))
    w = dict(WORKLOADS[args.workload])
    t0 = time.time()
    if w["kind"] == "uniform":
        w["n"] *= world
        rp, col = uniform_csr(w["n"], w["d"], w["seed"])
        dg = DeviceGraph.from_csr(rp, col, symmetric=True)
        del col
        desc = f"uniform (graph.py:30-43 process) n={w['n'] // 10**6}M (= 10M x {world} GPUs), max-degree {w['d']}"
    elif w["kind"] == "rmat":
        w["scale"] += int(round(math.log2(world)))
        dg = DeviceGraph.rmat(w["scale"], w["ef"], seed=w["seed"])
        rp, _ = dg.export()
        desc = f"R-MAT scale {w['scale']} (= base + log2 {world}), edge factor {w['ef']}, seed {w['seed']}"
    else:
        x, y, z = w["dims"]
        w["dims"] = (x, y, z * world)
        dg = DeviceGraph.mesh(*w["dims"])
        rp, _ = dg.export()
        desc = f"3-D 7-point mesh {x}x{y}x{z * world} (z-slabs)"
    gen_s = time.time() - t0
    m = dg.nnz // 2
    lo, hi = sh.balanced_ranges(rp, world)[rank]
    ops = sh.HipShard(dg, lo, hi)
    comm = sh.TorchTransport()

    def barrier():
        torch.cuda.synchronize()
        dist.barrier()

    for _ in range(max(args.warmup, 1)):
        res = sh.shard_color(ops, comm, want_colors=False)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):  # colours stay in HBM, as in the 1-GPU step
        res = sh.shard_color(ops, comm, want_colors=False)
    barrier()
    t = (time.perf_counter() - t0) / args.steps
    tt = torch.tensor([t], dtype=torch.float64, device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    line = None
    res.colors, _ = ops.colors(False)  # outside the timed region
    if rank == 0:
        unc, conf = dg.validate(res.colors)
        assert unc == 0 and conf == 0, f"invalid colouring: {unc} uncoloured, {conf} conflicts"
        one = dg.color("A", want_rounds=False, want_colors=True)  # reference run (outside timing)
        assert np.array_equal(one.colors, res.colors), "sharded colouring differs from the 1-GPU engine"
        balg = one.balg_bytes + 20.0 * dg.n + 8.0 * dg.nnz
        achieved = balg / world / t / 1e9
        line = {
            "metric": METRIC, "value": m / t, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": desc, "n": dg.n, "m_undirected": m, "nnz": dg.nnz, "max_degree": dg.max_degree,
                       "variant": "A (coloring.py)",
                       "parallelism": f"{world} vertex-range shards, round seams all-gathered over RCCL "
                                      "(deltas, or proposal-byte slices when denser)",
                       "rounds": res.rounds, "exchanges_per_step": res.exchanges,
                       "dense_exchanges_per_step": res.dense_exchanges, "jp_extra_sweeps": res.jp_sweeps,
                       "reseeds": res.reseeds, "graph_build_s": round(gen_s, 2)},
            "colors_used": res.max_color + 1,
            "roofline": {"bound": "hbm", "kernel": "whole colouring per GPU (sharded)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None},
            "whole_job_hbm_frac": achieved / HBM_PEAK_GBS,
            "cpu_baseline": None,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(s + "\n")
    ops.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="uniform10M", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--replicas", action="store_true",
                    help="N>1: colour N independent copies (one per GPU) instead of one sharded graph")
    ap.add_argument("--no-event-timing", action="store_true",
                    help="time the steps without per-launch HIP events (roofline fields then empty)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        # GC_BENCH_DEVICE pins every rank to one GPU (rehearsal of the multi-rank path on a
        # 1-GPU box, with GC_BENCH_BACKEND=gloo); the driver's runs use one GPU per rank
        dev = int(os.environ.get("GC_BENCH_DEVICE", local_rank))
        local_rank = dev
        torch.cuda.set_device(dev)
        backend = os.environ.get("GC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        if not args.replicas:
            return run_sharded(args, world, rank, local_rank, dist, torch)
    else:
        torch.cuda.set_device(0)

    from gcolor_amd import _native
    _native.check("gc_set_device", _native.load().gc_set_device(local_rank))
    w = WORKLOADS[args.workload]
    t0 = time.time()
    dg, host_csr = build_graph(w)
    gen_s = time.time() - t0
    m = dg.nnz // 2

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    # warmup; the last warmup step brackets every launch with HIP events to find the
    # dominant kernel class, whose launches alone are then event-timed in the timed region
    # (bracketing every launch costs ~30% of the step in inter-kernel gaps)
    probe = None
    for i in range(max(args.warmup, 1)):
        probe = dg.color("A", kernel_timing=(i == max(args.warmup, 1) - 1), want_rounds=False, want_colors=False)
    dom_class = max(((k, v) for k, v in probe.kernels.items() if v["bytes"] > 0), key=lambda kv: kv[1]["ms"])[0]
    barrier()
    # Timed region: K full colourings from the resident CSR.  Every launch is bracketed by
    # HIP events on the engine's own stream (kernel_timing), so the roofline numbers below
    # come from these same launches.
    kern = {}
    rounds = sweeps = reseeds = colours = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = dg.color("A", kernel_timing=None if args.no_event_timing else dom_class, want_rounds=False,
                     want_colors=False)
        for k, v in r.kernels.items():
            a = kern.setdefault(k, {"ms": 0.0, "launches": 0, "bytes": 0.0})
            a["ms"] += v["ms"]
            a["launches"] += v["launches"]
            a["bytes"] += v["bytes"]
        rounds, sweeps, reseeds, colours = r.rounds, r.jp_sweeps, r.reseeds, r.num_colors
    barrier()
    t = (time.perf_counter() - t0) / args.steps
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    for a in kern.values():
        a["ms"] /= args.steps
        a["launches"] //= args.steps
        a["bytes"] /= args.steps

    # validity of the colouring (outside the timed region)
    res = dg.color("A", want_colors=True, want_rounds=False)
    unc, conf = dg.validate()
    assert unc == 0 and (conf == 0 or not dg.symmetric), f"invalid colouring: {unc} uncoloured, {conf} conflicts"
    dom = (dom_class, kern[dom_class])
    achieved = dom[1]["bytes"] / (dom[1]["ms"] / 1e3) / 1e9 if dom[1]["ms"] > 0 else None
    balg = sum(v["bytes"] for v in kern.values()) + 20.0 * dg.n + 8.0 * dg.nnz
    traffic, traffic_src = pmc_traffic(dom[0], args.workload)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu, o = cpu_baseline(w, host_csr, dg)
        import numpy as np
        assert np.array_equal(o["colors"], res.colors), "GPU colouring differs from the oracle"
        cpu.pop("colors")
        cpu.pop("seconds")
    line = {
        "metric": METRIC,
        "value": world * m / t,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": w["desc"], "n": dg.n, "m_undirected": m, "nnz": dg.nnz,
                   "max_degree": dg.max_degree, "variant": "A (coloring.py)", "parallelism":
                   "replicas" if world > 1 else "single", "rounds": rounds, "jp_extra_sweeps": sweeps,
                   "reseeds": reseeds, "graph_build_s": round(gen_s, 2),
                   "event_timed_class": None if args.no_event_timing else dom_class},
        "colors_used": colours,
        "roofline": {"bound": "hbm", "kernel": dom[0], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": dom[1]["bytes"] / max(dom[1]["launches"], 1),
                     "avg_launch_ms": dom[1]["ms"] / max(dom[1]["launches"], 1),
                     "launches_per_step": dom[1]["launches"]},
        "whole_job_hbm_frac": balg / t / 1e9 / HBM_PEAK_GBS,
        "kernels_probe_step": {k: {"ms": round(v["ms"], 4), "launches": v["launches"], "GB": round(v["bytes"] / 1e9, 4)}
                               for k, v in probe.kernels.items() if v["launches"]},
        "cpu_baseline": cpu,
    }
    s = json.dumps(line)
    print(s, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(s + "\n")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
