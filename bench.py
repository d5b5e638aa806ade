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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="uniform10M", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
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

    for _ in range(args.warmup):
        dg.color("A", want_rounds=False, want_colors=False)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dg.color("A", want_rounds=False, want_colors=False)
    barrier()
    t = (time.perf_counter() - t0) / args.steps
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())

    # one instrumented step: per-kernel-class event timing + algorithmic bytes
    res = dg.color("A", kernel_timing=True, want_colors=True)
    unc, conf = dg.validate()
    assert unc == 0 and (conf == 0 or not dg.symmetric), f"invalid colouring: {unc} uncoloured, {conf} conflicts"
    dom = max(((k, v) for k, v in res.kernels.items() if v["bytes"] > 0), key=lambda kv: kv[1]["ms"])
    achieved = dom[1]["bytes"] / (dom[1]["ms"] / 1e3) / 1e9
    balg = res.balg_bytes + 20.0 * dg.n + 8.0 * dg.nnz

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
                   "replicas" if world > 1 else "single", "rounds": res.rounds, "jp_extra_sweeps": res.jp_sweeps,
                   "reseeds": res.reseeds, "graph_build_s": round(gen_s, 2)},
        "colors_used": res.num_colors,
        "roofline": {"bound": "hbm", "kernel": dom[0], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_step": dom[1]["bytes"], "kernel_ms_per_step": dom[1]["ms"],
                     "launches_per_step": dom[1]["launches"]},
        "whole_job_hbm_frac": balg / t / 1e9 / HBM_PEAK_GBS,
        "kernels": {k: {"ms": round(v["ms"], 4), "launches": v["launches"], "GB": round(v["bytes"] / 1e9, 4)}
                    for k, v in res.kernels.items() if v["launches"]},
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
