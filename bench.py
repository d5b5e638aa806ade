#!/usr/bin/env python3
"""Benchmark: edges coloured per second (TEPS) of the MI355X colouring engine.

Workload (default, BASELINE.json configs[2] = C3, the largest single-GPU config):
R-MAT scale 24, edge factor 16, (A,B,C) = (0.57,0.19,0.19), seed 1, self-loops dropped,
symmetrised, de-duplicated, generated on the device.  A step is SURVEY.md §8d's t: from a
CSR resident in HBM (rows in generation order) to a complete, validated colouring --
gc_graph_create_device (the rank partition of every row, coloring.py:64), gc_color (the hub
index is built inside; coloring.py:73-132 semantics, variant A unless --variant B),
gc_validate (coloring.py:149-162), gc_graph_destroy.  value = m / t (m = undirected edges =
nnz/2), whole job.  `recolour_ms` is the colouring alone on a persistent handle.
Other workloads (--workload): uniform10M (C2), rmat26 (north star), mesh512 (C4 on one
GPU), mesh256, uniform1M, rmat28 (C5, sharded runs).

Multi-GPU (bench.py --gpus N starts N ranks itself under torch.distributed.run, or runs as
one rank of an outside launcher): one process per GPU, ONE graph coloured by the ranks
together (gcolor_amd.shard: the hybrid by default), timed on the one-GPU step's definition
(create + colour + validate, MultiStep).  Default workload C5 (R-MAT-28, strong scaling);
--scaling weak grows the graph with N (uniform n x N, R-MAT scale + log2 N, mesh z x N).
Barrier + synchronize around the K timed steps, max time over ranks; value = m / t_max;
single_gpu_ms / speedup_vs_single_gpu: the same graph's one-GPU step on rank 0's GPU.

Extra objects on the JSON line:
  roofline      the kernel class that dominates the step BY TIME (every class, JP sweeps
                included), event-timed on the engine's stream over a second pass of the K
                steps right after the timed ones (`value` comes from the event-free pass,
                `roofline.event_pass_ms_per_step` is the second pass's wall time).
                achieved = SURVEY.md §8d algorithmic bytes / time when the class is credited
                any, else (the later JP sweeps: no §8d credit) the rocprofv3 FETCH+WRITE
                bytes of the class (profiles/pmc/<workload>.json) / time; `traffic` is the
                PMC bytes per launch.  `classes_probe_step` lists every class (probe step) and flags
                any whose algorithmic rate exceeds the HBM peak (bytes credited, not moved).
  whole_job_*   §8d bytes / t / peak (raw, and capped per class at what the peak could move
                in the class's time) and the physical fraction: rocprofv3 FETCH+WRITE bytes of
                every kernel of a timed step (--selected-regions run) / t / peak.
  north_star    R-MAT scale 26 on the same GPU, the same step (default run only).
  cpu_baseline  oracle/gcolor_omp.c, the multi-core C restatement (bit-exact with the
                oracle, tests/test_oracle_omp.py), on the box's host cores, rank 0 at N=1
"""
import argparse
import json
import math
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
    "rmat24": dict(kind="rmat", scale=24, ef=16, seed=1,
                   desc="C3: R-MAT scale 24, edge factor 16, (0.57,0.19,0.19), seed 1, symmetrised"),
    "rmat26": dict(kind="rmat", scale=26, ef=16, seed=1,
                   desc="north star: R-MAT scale 26, edge factor 16, (0.57,0.19,0.19), seed 1"),
    "rmat28": dict(kind="rmat", scale=28, ef=16, seed=1,
                   desc="C5: R-MAT scale 28, edge factor 16, (0.57,0.19,0.19), seed 1"),
    "uniform10M": dict(kind="uniform", n=10_000_000, d=16, seed=42,
                       desc="C2: uniform (graph.py:30-43 process) n=10M, max-degree 16, seed 42"),
    "mesh512": dict(kind="mesh", dims=(512, 512, 512), desc="C4: 3-D 7-point mesh 512^3"),
    "mesh256": dict(kind="mesh", dims=(256, 256, 256), desc="3-D 7-point mesh 256^3"),
    "uniform1M": dict(kind="uniform", n=1_000_000, d=16, seed=42, desc="uniform n=1M, max-degree 16"),
    "rmat20": dict(kind="rmat", scale=20, ef=16, seed=1, desc="R-MAT scale 20, edge factor 16, seed 1"),
}

# kernel names of each engine class (gc_stats.k_*), for the PMC bytes of the class
CLASS_KERNELS = {
    "init": ["k_init", "k_seed_prep"],
    "propose": ["k_propose", "k_propose_block"],
    # variant B's fold (k_b_init, its passes or the asynchronous fold) is its resolution class
    "resolve": ["k_resolve", "k_b_init", "k_b_ev", "k_b_adm", "k_b_async"],
    "sweep": ["k_sweep", "k_sweep_tail", "k_sweep_async"],
    "commit": ["k_commit", "k_commit_big", "k_pull", "k_b_commit", "k_hub_push_big"],
    "reseed": ["k_unc_compact", "k_cc_hook", "k_cc_best", "k_cc_seeds"],
    "other": ["k_close", "k_pack_c4", "k_fsort_count", "k_fsort_scan", "k_fsort_write", "k_front_count",
              "k_finalize", "k_stat_reduce", "k_b_reset", "k_b_fail0"],
}


def progress(msg):
    """A phase line on stderr (stdout carries only the JSON line): a long workload (R-MAT-28)
    otherwise writes nothing for minutes."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def build_graph(w):
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    if w["kind"] == "uniform":
        rp, col = uniform_csr(w["n"], w["d"], w["seed"])
        return DeviceGraph.from_csr(rp, col, symmetric=True), (rp, col)
    if w["kind"] == "rmat":
        return DeviceGraph.rmat(w["scale"], w["ef"], seed=w["seed"]), None
    return DeviceGraph.mesh(*w["dims"]), None


def resident_csr(dg, torch):
    """The input of the timed step ("from a resident CSR"): the graph's CSR as
    torch-owned HBM buffers, every row sorted by neighbour position -- the R-MAT generator's
    own row order, and an order the engine's rank partition does not produce (it lists
    lower-rank neighbours first), so each step partitions real input.  Built outside the
    timed region, chunked by rows to bound the sort's memory."""
    n, nnz = dg.n, dg.nnz
    d_rp = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    d_col = torch.empty(max(nnz, 1), dtype=torch.int32, device="cuda")
    dg.export_device(d_rp.data_ptr(), d_col.data_ptr())
    rp_h = d_rp.cpu().numpy()
    chunk = 1 << 27
    r = 0
    while r < n:
        r1 = int(np.searchsorted(rp_h, rp_h[r] + chunk, side="right")) - 1
        r1 = min(max(r1, r + 1), n)
        e0, e1 = int(rp_h[r]), int(rp_h[r1])
        if e1 > e0:
            deg = (d_rp[r + 1:r1 + 1] - d_rp[r:r1])
            rows = torch.repeat_interleave(torch.arange(r1 - r, device="cuda", dtype=torch.int64), deg)
            key = rows * n + d_col[e0:e1].to(torch.int64)
            key = torch.sort(key).values
            d_col[e0:e1] = (key % n).to(torch.int32)
            del rows, key, deg
        r = r1
    torch.cuda.synchronize()
    return d_rp, d_col


def pmc_file(workload, variant):
    return os.path.join(REPO, "profiles", "pmc", f"{workload}{'' if variant == 'A' else '_B'}.json")


def lib_sha16():
    """First 16 hex digits of sha256(libgcolor.so) -- the library gcolor_amd loads (GC_LIB_PATH for
    a variant build): the build a PMC summary describes."""
    import hashlib
    p = os.environ.get("GC_LIB_PATH") or os.path.join(PKG_DIR, "gcolor_amd", "lib", "libgcolor.so")
    if not os.path.exists(p):
        return None
    return hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]


def pmc_summary(workload, variant):
    """The rocprofv3 per-kernel summary of this bench command (tools/gpu_profile.sh), or None
    when it is missing or describes another build of libgcolor.so (counters of kernels that
    have since changed are not this build's traffic)."""
    p = pmc_file(workload, variant)
    if not os.path.exists(p):
        return None, None
    per = json.load(open(p))
    if per.get("_build") != lib_sha16():
        return None, os.path.relpath(p, REPO) + " (stale: another build; not used)"
    return per, os.path.relpath(p, REPO)


def pmc_class_bytes(workload, variant, key="hbm_bytes_per_launch"):
    """Per class: HBM bytes per launch of the class (FETCH_SIZE + WRITE_SIZE, KiB x 1024,
    summed over the class's kernels and divided by their launches) from the rocprofv3
    --pmc passes of this bench command (tools/gpu_profile.sh -> tools/pmc_summary.py);
    key="hbm_bytes_per_launch_calibrated": 2 x FETCH_SIZE + WRITE_SIZE (calibration())."""
    per, src = pmc_summary(workload, variant)
    if per is None:
        return {}, src
    out = {}
    for cls, names in CLASS_KERNELS.items():
        b = l = 0.0
        for k in names:
            e = per.get(k)
            if e and key in e:
                b += e[key] * e["launches"]
                l += e["launches"]
        if l:
            out[cls] = b / l
    return out, src


def calibration():
    """What rocprofv3's counters mean for this path's access patterns, measured on the box
    (tools/ubench/gather_bytes.hip -> profiles/calib/gather_bytes.json): FETCH_SIZE counts
    half of every line read -- 1/2 of a streaming read's bytes, 64 B per random 1-4 B gather
    whose line is 128 B -- and random 4-B gathers past the caches top out at `gather_Gops`
    (x 128 B: the HBM's achievable rate).  Calibrated HBM bytes = 2 x FETCH + WRITE."""
    p = os.path.join(REPO, "profiles", "calib", "gather_bytes.json")
    if not os.path.exists(p):
        return None
    c = json.load(open(p))
    g = c["k_gather4_big"]
    return {"source": os.path.relpath(p, REPO),
            "fetch_counted_over_streamed_bytes": c["k_stream_read16"]["fetch_over_named"],
            "fetch_counted_per_random_gather_B": g["fetch_bytes_per_op"],
            "write_counted_per_random_store_B": c["k_scatter4_big"]["write_bytes_per_op"],
            "gather_Gops": g["ops_per_s"] / 1e9,
            "gather_ceiling_GBps": g["ops_per_s"] * 2 * g["fetch_bytes_per_op"] / 1e9}


def cpu_baseline(w, host_csr, colors_gpu):
    """oracle/gcolor_omp.c (bit-exact restatement of the oracle) on every host core this
    process may use; TEPS of a full colouring of the same graph."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    rp, col = host_csr
    t0 = time.perf_counter()
    o = oracle.omp_color(rp, col, symmetric=True, threads=threads, want_rounds=False)
    dt = time.perf_counter() - t0
    m = len(col) / 2
    same = colors_gpu is not None and np.array_equal(o["colors"], colors_gpu)
    try:
        py = python_restatement()
    except Exception as e:  # context only: never lose the line over it
        py = {"error": repr(e)[:200]}
    return {"value": m / dt, "unit": "edges/s", "cores": threads, "kind": "port", "python_restatement": py,
            "sample": f"oracle/gcolor_omp.c (OpenMP, {threads} threads) colouring the full graph of {w['desc']} "
                      f"in {dt:.1f} s on {platform.processor() or platform.machine()} ({os.cpu_count()} CPUs "
                      f"visible); colours identical to the GPU's: {same}",
            "colors": int(o["max_color"]) + 1, "seconds": dt, "identical": same}


def cpu_baseline_sample(torch):
    """The N > 1 line's CPU baseline: the N = 1 workload (C3, R-MAT-24) as a bounded sample of
    the R-MAT family the N > 1 run colours (its R-MAT-28 would take minutes on the host), the GPU
    colouring of the same sample beside it for the identity check."""
    from gcolor_amd.engine import DeviceGraph
    w = WORKLOADS["rmat24"]
    with DeviceGraph.rmat(w["scale"], w["ef"], seed=w["seed"]) as dg:
        csr = dg.export()
        colors = dg.color("A").colors
    out = cpu_baseline(w, csr, colors)
    out["identical_to_gpu"] = bool(out.pop("identical"))
    out.pop("colors")
    out.pop("seconds")
    out["sample"] = "bounded sample (the N = 1 workload, same generator): " + out["sample"]
    return out


def python_restatement(scale=14):
    """Context for the CPU baseline: the oracle's pure-Python restatement (oracle.py py_color:
    the reference's per-vertex lambdas as Python loops, one thread, without Spark's overhead)
    on a bounded sample -- the same R-MAT generator at scale 14 -- checked against the C oracle."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(scale, 16, seed=1) as dg:
        rp, col = dg.export()
    adj = [col[rp[i]:rp[i + 1]].tolist() for i in range(len(rp) - 1)]
    t0 = time.perf_counter()
    o = oracle.py_color(adj, "A")
    dt = time.perf_counter() - t0
    same = np.array_equal(np.asarray(o["colors"], dtype=np.int32), oracle.c_color(rp, col, "A")["colors"])
    return {"value": len(col) / 2 / dt, "unit": "edges/s", "cores": 1, "seconds": round(dt, 3),
            "sample": f"R-MAT scale {scale} (edge factor 16, seed 1; {len(col) // 2} edges), oracle.py py_color, "
                      f"colours identical to the C oracle: {same}"}


class StepRunner:
    """The §8d step on one GPU, from a resident CSR ("device wall time from a
    resident CSR to a full valid colouring"): gc_graph_create_device (the rank partition of the
    input rows, coloring.py:64), gc_color (the hub index is built inside: a fresh handle has
    none), gc_validate (coloring.py:149-162), gc_graph_destroy."""

    def __init__(self, dg0, variant, mode, torch, barrier):
        self.V, self.mode, self.torch, self.barrier = variant, mode, torch, barrier
        self.n, self.nnz, self.max_degree, self.sym = dg0.n, dg0.nnz, dg0.max_degree, dg0.symmetric
        self.d_rp, self.d_col = resident_csr(dg0, torch)

    def recolour_ms(self, dg0, reps=2):
        return min(dg0.color(self.V, want_rounds=False, want_colors=False, **self.mode).device_ms
                   for _ in range(reps))

    def step(self, timing=None):
        from gcolor_amd.engine import DeviceGraph
        a = time.perf_counter()
        dg = DeviceGraph.from_device(self.d_rp.data_ptr(), self.d_col.data_ptr(), self.n, self.nnz, symmetric=self.sym,
                                     stream=self.torch.cuda.current_stream().cuda_stream)
        b = time.perf_counter()
        r = dg.color(self.V, kernel_timing=timing, want_rounds=False, want_colors=False, **self.mode)
        c = time.perf_counter()
        unc, conf = dg.validate()
        d = time.perf_counter()
        dg.close()
        e = time.perf_counter()
        assert unc == 0 and (conf == 0 or not self.sym), f"invalid colouring: {unc} uncoloured, {conf} conflicts"
        return r, {"create": b - a, "colour": c - b, "validate": d - c, "destroy": e - d}

    def steps(self, k, timing, roctx=False):
        kern, ph = {}, {}
        r = None
        self.barrier()
        if roctx:
            roctx_resume()
        t0 = time.perf_counter()
        for _ in range(k):
            r, p = self.step(timing)
            for key, v in r.kernels.items():
                a = kern.setdefault(key, {"ms": 0.0, "launches": 0, "bytes": 0.0})
                a["ms"] += v["ms"]
                a["launches"] += v["launches"]
                a["bytes"] += v["bytes"]
            for key, v in p.items():
                ph[key] = ph.get(key, 0.0) + v / k
        self.barrier()
        t = (time.perf_counter() - t0) / k
        if roctx:
            roctx_pause()
        for a in kern.values():
            a["ms"] /= k
            a["launches"] //= k
            a["bytes"] /= k
        return t, kern, r, ph

    def final_colouring(self):
        from gcolor_amd.engine import DeviceGraph
        with DeviceGraph.from_device(self.d_rp.data_ptr(), self.d_col.data_ptr(), self.n, self.nnz,
                                     symmetric=self.sym) as dg:
            res = dg.color(self.V, want_colors=True, want_rounds=False, **self.mode)
            unc, conf = dg.validate()
            assert unc == 0 and conf == 0
            return {"colors": res.colors, "csr": dg.export()}

    def end_to_end(self, rp, col, reps=2):
        """SURVEY.md §8d's "end-to-end time is also reported" (coloring.py:233-234's `Total
        execution time`, without file parsing): the CSR in host memory (pageable numpy) ->
        gc_graph_create (H2D + rank partition) -> gc_color -> gc_validate -> colours in host
        memory -> destroy.  Best of `reps`, outside the timed region; never `value`."""
        from gcolor_amd.engine import DeviceGraph
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            with DeviceGraph.from_csr(rp, col, symmetric=self.sym) as dg:
                res = dg.color(self.V, want_colors=True, want_rounds=False, **self.mode)
                unc, conf = dg.validate()
            dt = time.perf_counter() - t0
            assert unc == 0 and (conf == 0 or not self.sym) and len(res.colors) == self.n
            best = dt if best is None else min(best, dt)
        return best

    def close(self):
        self.d_rp = self.d_col = None
        self.torch.cuda.empty_cache()


_ROCTX = None


def _roctx():
    """rocprofv3 --selected-regions collects only between roctxProfilerResume/Pause: the
    profiling runs (tools/gpu_profile.sh) count the timed steps' kernels alone."""
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("GC_ROCTX"):
            import ctypes
            rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
            for name in (os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so.1"), "librocprofiler-sdk-roctx.so.1",
                         os.path.join(rocm, "lib", "libroctx64.so.4")):
                try:
                    _ROCTX = ctypes.CDLL(name)
                    break
                except OSError:
                    continue
    return _ROCTX


def roctx_resume():
    lib = _roctx()
    if lib:
        lib.roctxProfilerResume(0)


def roctx_pause():
    lib = _roctx()
    if lib:
        lib.roctxProfilerPause(0)


def capped_alg(kern, n, nnz):
    """§8d algorithmic bytes of a step with no class credited more than the HBM peak could
    move in that class's (event-timed) time, plus the validate pass."""
    tot = 0.0
    for v in kern.values():
        b = v["bytes"]
        if v["ms"] > 0:
            b = min(b, v["ms"] / 1e3 * HBM_PEAK_GBS * 1e9)
        tot += b
    return tot + 20.0 * n + 8.0 * nnz


def pmc_step_frac(workload, variant, t):
    """Physical fraction of the whole step: rocprofv3 FETCH_SIZE + WRITE_SIZE of every kernel
    of the timed steps (profiles/pmc/<workload>.json "_step", a --selected-regions run of this
    bench command) / t / peak -- as counted, and calibrated (2 x FETCH + WRITE, calibration())."""
    per, src = pmc_summary(workload, variant)
    st = per.get("_step") if per else None
    if not st or not st.get("steps"):
        return None
    b = st["bytes"] / st["steps"]
    out = {"bytes_per_step": b, "GBps": b / t / 1e9, "frac": b / t / 1e9 / HBM_PEAK_GBS, "source": src}
    if "fetch_bytes" in st:
        bc = (2 * st["fetch_bytes"] + st["write_bytes"]) / st["steps"]
        out.update({"bytes_per_step_calibrated": bc, "GBps_calibrated": bc / t / 1e9,
                    "frac_calibrated": bc / t / 1e9 / HBM_PEAK_GBS})
    return out


def north_star(torch, barrier, args):
    """BASELINE.json north_star's target graph, R-MAT scale 26 on one GPU, measured the same way
    (a few steps: it adds ~20 s to the default run)."""
    w = WORKLOADS["rmat26"]
    dg0, _ = build_graph(w)
    S = StepRunner(dg0, "A", {"priority": None, "speculative": False}, torch, barrier)
    dg0.close()
    probe, _ = S.step(timing=True)  # warmup; every class event-timed (for the capped fraction)
    t, kern, r, ph = S.steps(args.north_star_steps, None)
    m = S.nnz // 2
    balg = sum(v["bytes"] for v in kern.values()) + 20.0 * S.n + 8.0 * S.nnz
    out = {"workload": w["desc"], "n": S.n, "m_undirected": m, "steps": args.north_star_steps,
           "ms_per_step": t * 1e3, "edges_per_s": m / t, "colors_used": r.num_colors, "rounds": r.rounds,
           "async_jp_aborts": r.async_aborts, "hubs": r.hubs, "hubs_on": r.hubs > 0,
           "phases_ms": {k: round(v * 1e3, 3) for k, v in ph.items()},
           # §8d bytes / t / peak: a WORK ratio, not bandwidth -- §8d credits every hub proposal
           # with its whole row, which the pushed bitmaps never read (propose's class is above the
           # peak); the capped ratio credits no class more than the peak could move in its time
           "work_ratio": balg / t / 1e9 / HBM_PEAK_GBS,
           "work_ratio_capped": capped_alg(probe.kernels, S.n, S.nnz) / t / 1e9 / HBM_PEAK_GBS,
           "classes_probe_step": class_table(probe.kernels, pmc_class_bytes("rmat26", "A")[0]),
           # the physical figures: every kernel's bytes of a step (as counted, and calibrated:
           # 2 x FETCH + WRITE) / t / peak, and the dominant class on the calibrated basis
           "pmc_frac": pmc_step_frac("rmat26", "A", t),
           "roofline_calibrated": calibrated_roofline("rmat26", "A", probe.kernels)}
    # THE north-star figure: the whole step's HBM bytes on the calibrated basis
    # (2 x FETCH_SIZE + WRITE_SIZE of every kernel of a step, profiles/pmc/rmat26.json "_step",
    # the gfx950 correction of MI355X_MICROARCH.md) / this run's step time / 8 TB/s; null when
    # that summary is not of this build.  The as-counted figure stays beside it.
    pf = out["pmc_frac"]
    out["roofline_frac"] = pf.get("frac_calibrated") if pf else None
    out["roofline_frac_as_counted"] = pf.get("frac") if pf else None
    out["roofline_frac_basis"] = ("(2 x FETCH_SIZE + WRITE_SIZE per step, profiles/pmc/rmat26.json _step) / "
                                  "ms_per_step / 8 TB/s")
    S.close()
    return out


def variant_b_line(torch, barrier, args):
    """coloring_optimized.py's path (variant B) on the bench workload's graph (C3, R-MAT-24),
    the same §8d step, a few steps -- so the driver's own run measures it too.
    Its fold is the resolve class: roofline on the calibrated PMC basis of profiles/pmc/rmat24_B.json
    when that summary is of this build."""
    w = WORKLOADS["rmat24"]
    dg0, _ = build_graph(w)
    S = StepRunner(dg0, "B", {"priority": None, "speculative": False}, torch, barrier)
    dg0.close()
    probe, _ = S.step(timing=True)  # warmup, every class event-timed
    t, kern, r, ph = S.steps(args.variant_b_steps, None)
    m = S.nnz // 2
    out = {"workload": w["desc"], "variant": "B (coloring_optimized.py)", "steps": args.variant_b_steps,
           "ms_per_step": t * 1e3, "edges_per_s": m / t, "colors_used": r.num_colors, "rounds": r.rounds,
           "async_fold_aborts": r.async_aborts, "phases_ms": {k: round(v * 1e3, 3) for k, v in ph.items()},
           "roofline_calibrated": calibrated_roofline("rmat24", "B", probe.kernels),
           "pmc_frac": pmc_step_frac("rmat24", "B", t)}
    S.close()
    return out


def calibrated_roofline(workload, variant, kern):
    """The dominant class (by event-timed time) on the calibrated physical basis: 2 x FETCH_SIZE
    + WRITE_SIZE per launch (calibration()) / the class's average launch time, against the HBM
    peak and against the measured random-gather ceiling (what a gather-bound kernel can reach)."""
    cal = calibration()
    pmc_c, src = pmc_class_bytes(workload, variant, "hbm_bytes_per_launch_calibrated")
    timed = {k: v for k, v in kern.items() if v["launches"] and v["ms"] > 0}
    if not cal or not timed:
        return None
    cls = max(timed, key=lambda k: timed[k]["ms"])
    v = timed[cls]
    avg_ms = v["ms"] / v["launches"]
    out = {"kernel": cls, "kernels": CLASS_KERNELS.get(cls), "avg_launch_ms": avg_ms, "launches_per_step": v["launches"],
           "peak": HBM_PEAK_GBS, "gather_ceiling": cal["gather_ceiling_GBps"], "unit": "GB/s",
           "basis": "2 x FETCH_SIZE + WRITE_SIZE per launch (profiles/calib/gather_bytes.json)", "source": src}
    if cls in pmc_c:
        a = pmc_c[cls] / (avg_ms / 1e3) / 1e9
        out.update({"traffic": pmc_c[cls], "achieved": a, "frac": a / HBM_PEAK_GBS,
                    "frac_of_gather_ceiling": a / cal["gather_ceiling_GBps"]})
    return out


def class_table(kern, pmc):
    """Per class and step (the probe step: every class event-timed): ms, launches, §8d
    algorithmic GB and rate, PMC GB and rate (when a PMC summary exists)."""
    out = {}
    for k, v in kern.items():
        if not v["launches"]:
            continue
        e = {"ms": round(v["ms"], 4), "launches": v["launches"], "alg_GB": round(v["bytes"] / 1e9, 4)}
        if v["ms"] > 0:
            e["alg_GBps"] = round(v["bytes"] / v["ms"] / 1e6, 1)
            e["alg_frac"] = round(e["alg_GBps"] / HBM_PEAK_GBS, 4)
            if e["alg_frac"] > 1.0:  # credited bytes the path does not move (hub bitmaps): a work
                e["alg_over_peak"] = True  # ratio, not a bandwidth fraction
                e["work_ratio"] = e.pop("alg_frac")
        if k in pmc:
            e["pmc_GB"] = round(pmc[k] * v["launches"] / 1e9, 4)
            if v["bytes"] > 0:  # physical / algorithmic: > 1 is traffic the §8d model does not need
                e["pmc_over_alg"] = round(pmc[k] * v["launches"] / v["bytes"], 3)
            if v["ms"] > 0:
                e["pmc_GBps"] = round(pmc[k] * v["launches"] / v["ms"] / 1e6, 1)
                e["pmc_frac"] = round(e["pmc_GBps"] / HBM_PEAK_GBS, 4)
        out[k] = e
    return out


def scaled_workload(w, world, scaling):
    """The workload of an N-GPU run: --scaling weak grows it with N (uniform n x N, R-MAT scale
    + log2 N, mesh z x N), strong keeps it.  Returns (workload, description)."""
    w = dict(w)
    weak = scaling == "weak" and world > 1
    if w["kind"] == "uniform":
        if weak:
            w["n"] *= world
        desc = f"uniform (graph.py:30-43 process) n={w['n'] / 1e6:g}M, max-degree {w['d']}, seed {w['seed']}"
    elif w["kind"] == "rmat":
        if weak:
            w["scale"] += int(round(math.log2(world)))
        desc = f"R-MAT scale {w['scale']}, edge factor {w['ef']}, (0.57,0.19,0.19), seed {w['seed']}"
    else:
        x, y, z = w["dims"]
        if weak:
            w["dims"] = (x, y, z * world)
        desc = f"3-D 7-point mesh {x}x{y}x{w['dims'][2]}"
    w["desc"] = desc + (f" (= base x {world} GPUs)" if weak else "")
    return w


def replica_workload(w, world, rank):
    """--multi replicas: rank `rank`'s own base-size graph (seed + rank: independent colourings)."""
    w = scaled_workload(w, 1, "strong")
    if "seed" in w:
        w["seed"] += rank
    w["desc"] += f" (one per GPU, seed + rank, {world} independent colourings)"
    return w


def spawn_ranks(n):
    """`bench.py --gpus N` (N > 1) without a launcher: run this same command as N ranks under
    torch.distributed.run, one process per GPU, as a CHILD process -- this parent never touches
    the GPU and is not replaced (no exec) -- and return the child's exit status.  Rank 0 prints
    the JSON line; the ranks see WORLD_SIZE and do not spawn again."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    progress(f"--gpus {n}: starting {n} ranks (torch.distributed.run, 127.0.0.1:{port})")
    return subprocess.call(cmd)


class MultiStep:
    """The N-GPU step, on the ONE-GPU step's definition (SURVEY.md §8d's t): from the CSR
    resident in every rank's HBM to a complete, validated colouring of ONE graph.
      create    gc_graph_create_device (the rank partition of every row) + gc_shard_create (the
                rank's vertex range, its in-neighbour rows, the replicated hub state; the hub
                index is built inside)
      colour    hybrid_color: the rounds sharded over the ranks while the frontier is large
                (seams over RCCL), then every rank resumes the one-GPU engine from the replicated
                state (gcolor_amd.shard); --multi sharded: every round sharded
      validate  gc_validate_range over the rank's own vertex range + one all-reduce of the two
                counts (validate_graph_coloring, coloring.py:149-162, split by rows)
      destroy   both handles
    The reference's counterpart is its partitioned execution (coloring.py:190-209: local[*],
    parallelize, partitionBy) and the distributed count of coloring.py:149-162."""

    def __init__(self, args, w, world, rank, comm, torch, dist):
        from gcolor_amd import shard as sh
        self.args, self.world, self.rank, self.comm, self.torch, self.dist = args, world, rank, comm, torch, dist
        self.sh = sh
        dg0, _ = build_graph(w)  # every rank generates the same graph (deterministic, on its own GPU)
        if rank == 0:
            progress(f"rank 0: graph generated ({dg0.n} vertices, {dg0.nnz} entries)")
        self.n, self.nnz, self.max_degree, self.sym = dg0.n, dg0.nnz, dg0.max_degree, dg0.symmetric
        rp, _ = dg0.export(col=False)
        self.ranges = sh.balanced_ranges(rp, world)
        self.lo, self.hi = self.ranges[rank]
        del rp
        self.d_rp, self.d_col = resident_csr(dg0, torch)
        dg0.close()
        if rank == 0:
            progress("rank 0: resident CSR ready")
        self.hybrid = args.multi == "hybrid"
        self.switch_below = args.switch_below if args.switch_below > 0 else max(4096, self.n // 64)

    def colour(self, ops, dg, want_colors):
        sh = self.sh
        kw = dict(want_colors=want_colors, ahead=self.args.seam_ahead, inline_max=self.args.seam_inline_max)
        if self.hybrid:
            return sh.hybrid_color(ops, self.comm, sh.engine_resume(dg), self.switch_below, switch_after_peak=True, **kw)
        return sh.shard_color(ops, self.comm, **kw)

    def step(self, want_colors=False):
        from gcolor_amd.engine import DeviceGraph
        torch = self.torch
        a = time.perf_counter()
        dg = DeviceGraph.from_device(self.d_rp.data_ptr(), self.d_col.data_ptr(), self.n, self.nnz, symmetric=self.sym,
                                     stream=torch.cuda.current_stream().cuda_stream)
        ops = self.sh.HipShard(dg, self.lo, self.hi)
        b = time.perf_counter()
        res = self.colour(ops, dg, want_colors)
        c = time.perf_counter()
        if res.switch_round is not None:  # the resumed engine holds the colouring on every rank
            unc, conf = dg.validate(None, lo=self.lo, hi=self.hi)
        else:  # finished sharded: the shard's colours
            cols = res.colors if res.colors is not None else ops.colors(False, True)[0]
            unc, conf = dg.validate(cols, lo=self.lo, hi=self.hi)
        cnt = torch.tensor([unc, conf], dtype=torch.int64, device="cuda" if self.comm.backend == "nccl" else "cpu")
        self.dist.all_reduce(cnt)
        unc, conf = (int(x) for x in cnt.tolist())
        d = time.perf_counter()
        ops.close()
        dg.close()
        e = time.perf_counter()
        assert unc == 0 and (conf == 0 or not self.sym), f"invalid colouring: {unc} uncoloured, {conf} conflicts"
        return res, {"create": b - a, "colour": c - b, "validate": d - c, "destroy": e - d}

    def single_gpu(self, reps=2):
        """The same graph's ONE-GPU step (the N = 1 line's definition) on this rank's GPU: the
        best of `reps` step times, the colours (a first, untimed run) and one event-timed probe
        (its kernel classes, for the roofline)."""
        from gcolor_amd.engine import DeviceGraph
        times, colours, probe = [], None, None
        for i in range(reps + 2):  # 0: colours to host; 1..reps: timed; last: event-timed probe
            timing = i == reps + 1
            a = time.perf_counter()
            with DeviceGraph.from_device(self.d_rp.data_ptr(), self.d_col.data_ptr(), self.n, self.nnz,
                                         symmetric=self.sym) as dg:
                r = dg.color("A", want_rounds=False, want_colors=(i == 0), kernel_timing=timing)
                unc, conf = dg.validate()
            dt = time.perf_counter() - a
            assert unc == 0 and conf == 0, f"invalid one-GPU colouring: {unc} uncoloured, {conf} conflicts"
            if i == 0:
                colours = r.colors
            elif timing:
                probe = r
            else:
                times.append(dt)
        return min(times), colours, probe

    def close(self):
        self.d_rp = self.d_col = None
        self.torch.cuda.empty_cache()


def run_multi(args, world, rank, local_rank, dist, torch):
    """N > 1 (or --sharded at N = 1): ONE graph coloured by the N ranks together, timed on the
    N = 1 step's definition (MultiStep).  value = m / t_max, whole job."""
    from gcolor_amd import _native
    from gcolor_amd import shard as sh
    _native.check("gc_set_device", _native.load().gc_set_device(local_rank))
    w = scaled_workload(WORKLOADS[args.workload], world, args.scaling)
    t0 = time.time()
    if rank == 0:
        progress(f"building {args.workload} ({world} ranks)")
    comm = sh.TorchTransport()
    S = MultiStep(args, w, world, rank, comm, torch, dist)
    gen_s = time.time() - t0
    m = S.nnz // 2
    if rank == 0:
        progress(f"graph and resident CSR ready in {gen_s:.1f} s; warmup")

    def barrier():
        torch.cuda.synchronize()
        dist.barrier()

    for i in range(max(args.warmup, 1)):
        a = time.perf_counter()
        res, _ = S.step(False)
        if rank == 0:
            progress(f"warmup step {i}: {(time.perf_counter() - a) * 1e3:.1f} ms (switch at round {res.switch_round})")
    if rank == 0:
        progress("warmup done; timed steps")
    barrier()
    t0 = time.perf_counter()
    ph = {}
    for _ in range(args.steps):  # colours stay in HBM, as in the 1-GPU step
        res, p = S.step(False)
        for k, v in p.items():
            ph[k] = ph.get(k, 0.0) + v / args.steps
    barrier()
    t = (time.perf_counter() - t0) / args.steps
    tt = torch.tensor([t], dtype=torch.float64, device="cuda" if comm.backend == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    if rank == 0:
        progress(f"timed steps done ({t * 1e3:.1f} ms per step); the one-GPU step of the same graph")
    res, _ = S.step(True)  # once more with the colours to host, outside the timed region
    line = None
    if rank == 0:
        t1, one_colours, probe = S.single_gpu()  # the same graph, the N = 1 step, on rank 0's GPU
        assert np.array_equal(one_colours, res.colors), "multi-GPU colouring differs from the one-GPU engine"
        cap = capped_alg(probe.kernels, S.n, S.nnz)
        achieved = cap / world / t / 1e9
        # traffic: the same graph's one-GPU step's HBM bytes (rocprofv3, calibrated 2 x FETCH +
        # WRITE, profiles/pmc/<workload>.json of this build) split over the N ranks -- the
        # ranks' own counters are not collected (rocprofv3 runs one process); null when stale
        one_pmc = pmc_step_frac(args.workload, "A", t1) if w["desc"] == WORKLOADS[args.workload]["desc"] else None
        step_bytes = one_pmc and one_pmc.get("bytes_per_step_calibrated")
        phys = ({"traffic": step_bytes / world, "achieved": step_bytes / world / t / 1e9,
                 "frac": step_bytes / world / t / 1e9 / HBM_PEAK_GBS, "source": one_pmc["source"],
                 "basis": "the one-GPU step's calibrated HBM bytes per step / N / t"} if step_bytes else None)
        cpu = None
        if not args.no_cpu_baseline:
            try:  # a bounded sample of the same R-MAT family: C3 (R-MAT-24), ~10 s on 16 threads
                progress("CPU baseline (bounded sample: R-MAT-24)")
                cpu = cpu_baseline_sample(torch)
            except Exception as e:  # noqa: BLE001 -- a failing baseline is reported, not the line lost
                cpu = {"error": f"{type(e).__name__}: {e}"}
        line = {
            "metric": METRIC, "value": m / t, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t * 1e3, "higher_is_better": True,
            "scaling": args.scaling if world > 1 else None,
            "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": w["desc"], "n": S.n, "m_undirected": m, "nnz": S.nnz, "max_degree": S.max_degree,
                       "variant": "A (coloring.py)",
                       "parallelism": f"{world} vertex-range shards (balanced by deg+1), round seams over "
                                      f"{'RCCL' if comm.backend == 'nccl' else comm.backend}"
                                      + (f"; hybrid: from the first round with a frontier below {S.switch_below}, once "
                                         f"the frontier has reached it (or after {sh.SWITCH_GRACE} rounds), every rank "
                                         f"finishes on its own one-GPU engine" if S.hybrid else ""),
                       "multi": "hybrid" if S.hybrid else "sharded", "switch_round": res.switch_round,
                       "step": "the one-GPU step's definition: resident CSR (HBM, every rank) -> gc_graph_create_device "
                               "(rank partition) + gc_shard_create (hub index inside) -> colouring over the ranks -> "
                               "gc_validate_range of each rank's vertex range + all-reduce -> destroy",
                       "rounds": res.rounds, "exchanges_per_step": res.exchanges,
                       "dense_exchanges_per_step": res.dense_exchanges, "jp_extra_sweeps": res.jp_sweeps,
                       "reseeds": res.reseeds, "graph_build_s": round(gen_s, 2),
                       "seam_ahead": args.seam_ahead, "seam_inline_max": args.seam_inline_max,
                       "sweep_seams_run_ahead": res.ahead_seams, "fused_misses": res.fused_misses,
                       "hubs": probe.hubs, "hubs_on": probe.hubs > 0,
                       # the same graph, the N = 1 step (create + colour + validate), rank 0's GPU, best of 2
                       "single_gpu_ms": round(t1 * 1e3, 2), "speedup_vs_single_gpu": round(t1 / t, 3)},
            "phases_ms": {k: round(v * 1e3, 3) for k, v in ph.items()},
            "colors_used": res.max_color + 1,
            "roofline": {"bound": "hbm", "kernel": "whole step per GPU",
                         "achieved": phys["achieved"] if phys else achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (phys["achieved"] if phys else achieved) / HBM_PEAK_GBS,
                         "achieved_basis": (phys["basis"] + f" ({phys['source']})") if phys else
                         "§8d algorithmic bytes of the one-GPU colouring (no class credited above the peak) / N / t "
                         "(no rocprofv3 summary of this build)",
                         "traffic": phys["traffic"] if phys else None,
                         "algorithmic": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS}},
            "cpu_baseline": cpu,
        }
    barrier()  # every rank waits for rank 0's one-GPU reference
    S.close()
    if line is not None:
        s = json.dumps(line)
        print(s, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(s + "\n")
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: rmat24 (C3) on one GPU; rmat28 (C5, the north star's scaling graph) for the "
                         "modes that split one colouring over N > 1 GPUs (hybrid, sharded)")
    ap.add_argument("--no-variant-b", action="store_true",
                    help="skip the variant-B (coloring_optimized.py) measurement the default run adds (variant_b object)")
    ap.add_argument("--variant-b-steps", type=int, default=3)
    ap.add_argument("--variant", default="A", choices=["A", "B"],
                    help="A = coloring.py semantics, B = coloring_optimized.py ('Optimizovano')")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="N > 1: weak grows the graph with N, strong keeps the workload's graph (default: strong "
                         "for the modes that split one colouring -- hybrid, sharded -- weak for replicated / replicas)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--multi", default="hybrid", choices=["replicated", "replicas", "sharded", "hybrid"],
                    help="N>1: hybrid (default) -- one graph, sharded rounds while the frontier is large, then every "
                         "rank resumes the one-GPU engine from the replicated state (gcolor_amd.shard.hybrid_color; "
                         "DESIGN.md §7); replicated -- every rank runs the one-GPU engine on the whole graph, no "
                         "exchange, the job's time is the slowest rank's; replicas -- N independent colourings, one "
                         "base-size graph per rank (seed + rank), value = all ranks' edges / the slowest rank's time "
                         "(throughput of many graphs, not of one); sharded -- one graph cut into vertex-range "
                         "shards with round seams over RCCL in every round (gcolor_amd.shard; DESIGN.md §7)")
    ap.add_argument("--switch-below", type=int, default=0,
                    help="hybrid: frontier size below which the ranks switch to the one-GPU engine "
                         "(0: max(4096, n / 64))")
    ap.add_argument("--priority-seed", type=int, default=None,
                    help="north_star mode N1: JP rounds ranked by prio_hash(seed, v) instead of (deg, pos)")
    ap.add_argument("--speculative", action="store_true",
                    help="north_star mode N1: speculative first-fit rounds with one-shot resolution")
    ap.add_argument("--sharded", action="store_true",
                    help="run the sharded engine even at N=1 (one-rank RCCL group): the multi-GPU protocol's "
                         "own cost on one GPU, against the single-GPU engine on the same graph")
    ap.add_argument("--seam-ahead", type=int, default=4,
                    help="sharded runs: JP sweep seams a fused round runs ahead of the host (gcolor_amd.shard)")
    ap.add_argument("--seam-inline-max", type=int, default=1 << 16,
                    help="sharded runs: largest inline delta part of a seam (gcolor_amd.shard)")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the R-MAT-26 measurement the default run adds (north_star object)")
    ap.add_argument("--north-star-steps", type=int, default=3)
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the end-to-end measurement (host CSR -> colours on host) the N=1 line adds")
    ap.add_argument("--no-event-timing", action="store_true",
                    help="time the steps without per-launch HIP events (roofline fields then empty)")
    args = ap.parse_args()
    if args.scaling is None:
        args.scaling = "strong" if args.multi in ("hybrid", "sharded") else "weak"
    if args.workload is None:
        args.workload = "rmat28" if args.gpus > 1 and args.multi in ("hybrid", "sharded") else "rmat24"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:  # no launcher: start the N ranks ourselves
        sys.exit(spawn_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started {world} ranks (WORLD_SIZE)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU: the library may park all but 48 GB of HBM between steps (a large
    # handle's destroy otherwise frees ~40 GB that the next step's hipMalloc waits seconds for,
    # csrc/gc_alloc.hip).  Not when ranks share one GPU (GC_BENCH_DEVICE rehearsals): the
    # library's conservative 64 GB default then stays.
    if "GC_BENCH_DEVICE" not in os.environ:
        os.environ.setdefault("GC_ALLOC_IDLE_RESERVE_GB", "48")
    import torch
    dist = None
    if world == 1 and args.sharded:  # a one-rank group without a launcher
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.sharded:
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
        if args.sharded or args.multi in ("sharded", "hybrid"):
            return run_multi(args, world, rank, local_rank, dist, torch)
    else:
        torch.cuda.set_device(0)

    from gcolor_amd import _native
    _native.check("gc_set_device", _native.load().gc_set_device(local_rank))
    replicas = world > 1 and args.multi == "replicas"
    w = replica_workload(WORKLOADS[args.workload], world, rank) if replicas else \
        scaled_workload(WORKLOADS[args.workload], world, args.scaling)
    V = args.variant
    # north_star N1 modes (variant A only): seeded priorities / speculative first-fit
    mode = {"priority": args.priority_seed, "speculative": args.speculative}
    if V == "B" and (args.priority_seed is not None or args.speculative):
        raise SystemExit("--priority-seed / --speculative are variant A modes")
    t0 = time.time()
    progress(f"building {args.workload}")
    dg0, host_csr = build_graph(w)
    progress("graph built")
    gen_s = time.time() - t0

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    S = StepRunner(dg0, V, mode, torch, barrier)
    info = {"n": S.n, "nnz": S.nnz, "max_degree": S.max_degree}
    m = S.nnz // 2
    recolour_ms = S.recolour_ms(dg0)  # the same graph kept resident (round 2's step), for reference
    dg0.close()
    # warmup; the last warmup step brackets every launch with HIP events to find the class
    # that dominates by time, whose launches alone are then event-timed in the timed region
    # (bracketing every launch costs ~30% of the step in inter-kernel gaps)
    probe = None
    for i in range(max(args.warmup, 1)):
        probe, _ = S.step(timing=(i == max(args.warmup, 1) - 1))
    dom_class = max(probe.kernels.items(), key=lambda kv: kv[1]["ms"])[0]
    # Timed region: K full steps: resident CSR -> graph with its rank
    # partition -> colouring (hub index built inside) -> validation -> handle released, no
    # events.  Then the same K steps again with the dominant class's launch runs bracketed by
    # HIP events on the engine's own stream (the roofline's launch durations).
    progress("warmup done; timed steps")
    t, kern, r, phases = S.steps(args.steps, None, roctx=True)
    progress(f"timed steps done ({t * 1e3:.1f} ms per step)")
    t_self = t  # this rank's own step time: for replicated runs, the one-GPU time of the same work
    rounds, sweeps, reseeds, colours = r.rounds, r.jp_sweeps, r.reseeds, r.num_colors
    m_all = m  # edges coloured per step by the whole job
    if dist is not None:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
        if replicas:  # every rank coloured its own graph
            mm = torch.tensor([float(m)], dtype=torch.float64, device="cuda")
            dist.all_reduce(mm, op=dist.ReduceOp.SUM)
            m_all = float(mm.item())
    t_ev = None
    if not args.no_event_timing:
        t_ev, kern, _, _ = S.steps(args.steps, dom_class)

    pmc, pmc_src = pmc_class_bytes(args.workload, V)
    dom = kern[dom_class]
    launches = max(dom["launches"], 1)
    avg_ms = dom["ms"] / launches
    alg_per_launch = dom["bytes"] / launches
    traffic_counted = pmc.get(dom_class)
    alg_rate = alg_per_launch / (avg_ms / 1e3) / 1e9 if dom["ms"] > 0 else 0.0
    balg = sum(v["bytes"] for v in kern.values()) + 20.0 * S.n + 8.0 * S.nnz
    cal_roof = None
    pmc_c, _ = pmc_class_bytes(args.workload, V, "hbm_bytes_per_launch_calibrated")
    cal = calibration()
    if cal and dom_class in pmc_c and dom["ms"] > 0:
        a = pmc_c[dom_class] / (avg_ms / 1e3) / 1e9
        cal_roof = {"achieved": a, "frac": a / HBM_PEAK_GBS, "traffic": pmc_c[dom_class],
                    "gather_ceiling": cal["gather_ceiling_GBps"], "frac_of_gather_ceiling": a / cal["gather_ceiling_GBps"]}
    # The headline figure: the dominant class's HBM bytes per launch on the
    # calibrated physical basis -- 2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950
    # correction, from a rocprofv3 summary of THIS build -- / its event-timed launch time.  The
    # as-counted PMC rate and the §8d algorithmic rate stay beside it.
    as_counted = ({"achieved": traffic_counted / (avg_ms / 1e3) / 1e9,
                   "frac": traffic_counted / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": traffic_counted}
                  if traffic_counted is not None and dom["ms"] > 0 else None)
    algorithmic = ({"achieved": alg_rate, "frac": alg_rate / HBM_PEAK_GBS, "bytes_per_launch": alg_per_launch,
                    "over_peak": alg_rate > HBM_PEAK_GBS} if alg_per_launch > 0 and dom["ms"] > 0 else None)
    if cal_roof is not None:
        basis, achieved, traffic = ("rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch (calibrated, "
                                    "profiles/calib/gather_bytes.json)"), cal_roof["achieved"], cal_roof["traffic"]
    elif algorithmic is not None and not algorithmic["over_peak"]:
        basis, achieved, traffic = "algorithmic (SURVEY.md §8d): no rocprofv3 summary of this build", alg_rate, None
    elif as_counted is not None:
        basis, achieved, traffic = "rocprofv3 FETCH_SIZE+WRITE_SIZE as counted (no calibration file)", \
            as_counted["achieved"], traffic_counted
    else:
        basis = ("unmeasured: " + ("the class has no §8d credit" if alg_per_launch <= 0 else
                 "§8d credit above the HBM peak (hub bitmaps stand in for rows)") +
                 " and no rocprofv3 summary of this build (profiles/pmc)")
        achieved, traffic = None, None

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    cpu = None
    final = None
    if world == 1 and not args.no_cpu_baseline and V == "A" and args.priority_seed is None and not args.speculative:
        final = S.final_colouring()  # outside the timed region
        try:
            progress("CPU baseline")
            cpu = cpu_baseline(w, host_csr or final["csr"], final["colors"])
            # the colours must equal the restatement's (bit-exact semantics); a difference is
            # reported in the line (identical_to_gpu) rather than losing the measurement
            cpu["identical_to_gpu"] = bool(cpu.pop("identical"))
            if not cpu["identical_to_gpu"]:
                print("WARNING: GPU colouring differs from the CPU restatement", file=sys.stderr, flush=True)
            cpu.pop("colors")
            cpu.pop("seconds")
        except Exception as e:  # noqa: BLE001 -- a failing baseline is reported, not the line lost
            cpu = {"error": f"{type(e).__name__}: {e}"}
            print(f"WARNING: cpu_baseline failed: {cpu['error']}", file=sys.stderr, flush=True)
    e2e = None
    if world == 1 and not args.no_end_to_end:
        try:
            csr = host_csr or (final["csr"] if final else S.final_colouring()["csr"])
            progress("end to end")
            e2e_s = S.end_to_end(*csr)
            e2e = {"ms": round(e2e_s * 1e3, 3), "edges_per_s": m / e2e_s,
                   "path": "CSR in pageable host memory -> gc_graph_create (H2D + rank partition) -> gc_color -> "
                           "gc_validate -> colours in host memory -> destroy (best of 2; coloring.py:233-234 "
                           "without the JSON parse)"}
            del csr
        except Exception as e:  # noqa: BLE001 -- context only
            e2e = {"error": f"{type(e).__name__}: {e}"}
    final = None
    ns = None
    if world == 1 and args.workload == "rmat24" and not args.no_north_star and V == "A" and not any(mode.values()):
        S.close()
        try:
            progress("north star (R-MAT-26)")
            ns = north_star(torch, barrier, args)
        except Exception as e:  # noqa: BLE001 -- reported in the line, which still prints
            ns = {"error": f"{type(e).__name__}: {e}"}
            print(f"WARNING: north_star failed: {ns['error']}", file=sys.stderr, flush=True)
    vb = None
    if world == 1 and args.workload == "rmat24" and not args.no_variant_b and V == "A" and not any(mode.values()):
        try:
            progress("variant B (R-MAT-24)")
            vb = variant_b_line(torch, barrier, args)
        except Exception as e:  # noqa: BLE001 -- reported in the line, which still prints
            vb = {"error": f"{type(e).__name__}: {e}"}
            print(f"WARNING: variant_b failed: {vb['error']}", file=sys.stderr, flush=True)
    classes = class_table(probe.kernels, pmc)
    line = {
        "metric": METRIC,
        "value": m_all / t,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling if world > 1 else None,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": w["desc"], "n": info["n"], "m_undirected": m, "nnz": info["nnz"],
                   "max_degree": info["max_degree"], "variant": "A (coloring.py)" if V == "A" else
                   "B (coloring_optimized.py)",
                   "parallelism": ((f"replicas: {world} independent colourings, one graph per rank, no exchange; "
                                    "value = all ranks' edges / the slowest rank's time") if replicas else
                                   (f"replicated: each of the {world} ranks runs the one-GPU engine on the whole graph, "
                                    "no exchange (the rounds are a latency chain: DESIGN.md §7); time = slowest rank"))
                                  if world > 1 else "single",
                   # every N > 1 line states the one-GPU time of its work: rank 0's own step time
                   # (replicated: the same graph; replicas: rank 0's own graph)
                   "single_gpu_ms": round(t_self * 1e3, 3) if world > 1 else None,
                   "speedup_vs_single_gpu": round(t_self / t, 3) if world > 1 else None,
                   "rank": ("(deg, pos) (coloring.py:64)" if args.priority_seed is None
                            else f"prio_hash(seed={args.priority_seed}, v), pos"),
                   "resolution": "speculative first-fit, one-shot" if args.speculative else "Jones-Plassmann LFMIS",
                   "step": "resident CSR (HBM, rows in generation order) -> gc_graph_create_device (rank "
                           "partition) -> gc_color (hub index built inside) -> gc_validate -> destroy",
                   "rounds": rounds, "jp_extra_sweeps": sweeps, "reseeds": reseeds,
                   "async_jp_aborts": r.async_aborts,
                   # the hub engine (pushed forbidden-colour bitmaps, hub JP): a graph with hubs whose
                   # index did not fit runs row scans instead (gc_color warns on stderr)
                   "hubs": r.hubs, "hubs_on": r.hubs > 0,
                   "graph_build_s": round(gen_s, 2),
                   "event_timed_class": None if args.no_event_timing else dom_class},
        "end_to_end_ms": e2e and e2e.get("ms"),
        "end_to_end": e2e,
        "colors_used": colours,
        "phases_ms": {k: round(v * 1e3, 3) for k, v in phases.items()},
        "recolour_ms": round(recolour_ms, 3),
        "roofline": {"bound": "hbm", "kernel": dom_class, "kernels": CLASS_KERNELS.get(dom_class),
                     "achieved": achieved, "achieved_basis": basis, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                     "traffic_source": pmc_src and f"{pmc_src} (HBM bytes per launch, 2 x FETCH_SIZE + WRITE_SIZE)",
                     "as_counted": as_counted, "algorithmic": algorithmic,
                     "algorithmic_bytes_per_launch": alg_per_launch, "avg_launch_ms": avg_ms,
                     "launches_per_step": dom["launches"],
                     "share_of_step": dom["ms"] / (t_ev * 1e3) if t_ev else None,
                     "event_pass_ms_per_step": t_ev and t_ev * 1e3,
                     # the same class on the calibrated basis (2 x FETCH + WRITE: FETCH_SIZE counts
                     # half of every line read, profiles/calib/gather_bytes.json)
                     "calibrated": cal_roof},
        "calibration": calibration(),
        "classes_probe_step": classes,
        # whole job, §8d algorithmic bytes / t: a work-efficiency ratio against the peak, NOT
        # bandwidth (hub bitmaps skip row reads §8d credits); the capped figure credits no class
        # more bytes than the peak could move in its time
        "whole_job_work_ratio": balg / t / 1e9 / HBM_PEAK_GBS,
        "whole_job_work_ratio_capped": capped_alg(probe.kernels, info["n"], info["nnz"]) / t / 1e9
                                        / HBM_PEAK_GBS,
        "whole_job_pmc_frac": pmc_step_frac(args.workload, V, t),
        "north_star": ns,
        "variant_b": vb,
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
