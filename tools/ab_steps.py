#!/usr/bin/env python3
"""Interleaved A/B of environment knobs inside ONE process on one GPU: the §8d step (resident
CSR -> gc_graph_create_device -> gc_color -> gc_validate -> destroy) of one workload, run
round-robin over the configurations (A, B, C, A, B, C, ...) so that box-to-box and drift
effects fall on every configuration alike.  Every configuration's colouring must equal the
first one's (colours, rounds): a knob that changes the result is reported and stops the run.

  python tools/ab_steps.py WORKLOAD REPS NAME=VAR:val+VAR:val ...   ("base" = no variables)
  e.g. tools/ab_steps.py rmat24 5 base c8=GC_VALIDATE_C8:1

Prints one line per step and a summary (median / min ms per configuration, and the median's
ratio to the first configuration).  Compile-time variants need a process each (GC_LIB_PATH).
"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))


def parse(specs):
    out = []
    for s in specs:
        name, _, rest = s.partition("=")
        env = {}
        for kv in filter(None, rest.split("+")):
            k, _, v = kv.partition(":")
            env[k] = v
        out.append((name, env))
    return out


def main():
    import numpy as np
    import torch
    import bench
    from gcolor_amd.engine import DeviceGraph
    wl, reps, cfgs = sys.argv[1], int(sys.argv[2]), parse(sys.argv[3:] or ["base"])
    variant = os.environ.get("AB_VARIANT", "A")
    torch.cuda.set_device(0)
    dg0, _ = bench.build_graph(bench.WORKLOADS[wl])
    d_rp, d_col = bench.resident_csr(dg0, torch)
    n, nnz, sym = dg0.n, dg0.nnz, dg0.symmetric
    dg0.close()
    keys = sorted({k for _, e in cfgs for k in e})
    base_env = {k: os.environ.get(k) for k in keys}

    def set_env(env):
        for k in keys:
            v = env.get(k, base_env[k])
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    def step(want_colors):
        torch.cuda.synchronize()
        a = time.perf_counter()
        dg = DeviceGraph.from_device(d_rp.data_ptr(), d_col.data_ptr(), n, nnz, symmetric=sym)
        r = dg.color(variant, want_rounds=False, want_colors=want_colors)
        unc, conf = dg.validate()
        dg.close()
        dt = time.perf_counter() - a
        assert unc == 0 and (conf == 0 or not sym), (unc, conf)
        return dt, r

    ref = None
    for name, env in cfgs:  # warm up every configuration once, checking its colouring
        set_env(env)
        _, r = step(True)
        sig = (r.rounds, r.num_colors)
        if ref is None:
            ref = (sig, r.colors)
        elif sig != ref[0] or not np.array_equal(r.colors, ref[1]):
            print(f"{name}: colouring differs from {cfgs[0][0]} ({sig} vs {ref[0]})", flush=True)
            sys.exit(1)
        print(f"{wl} {name} warm: rounds {r.rounds} colours {r.num_colors} device {r.device_ms:.2f} ms", flush=True)
    times = {name: [] for name, _ in cfgs}
    for i in range(reps):
        for name, env in cfgs:
            set_env(env)
            dt, r = step(False)
            times[name].append(dt * 1e3)
            print(f"{wl} rep {i} {name}: {dt * 1e3:.2f} ms (device colour {r.device_ms:.2f})", flush=True)
    set_env({})
    m0 = statistics.median(times[cfgs[0][0]])
    print(f"== {wl} ({n} vertices, {nnz // 2} edges), {reps} interleaved reps, variant {variant}")
    for name, env in cfgs:
        ts = times[name]
        md = statistics.median(ts)
        print(f"== {name:>16}: median {md:8.2f} ms  min {min(ts):8.2f}  ratio {md / m0:.4f}  {env}", flush=True)


if __name__ == "__main__":
    main()
