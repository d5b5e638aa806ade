#!/usr/bin/env python3
"""Phase timing of the §8d step on one GPU: resident CSR -> graph (rank partition) ->
colouring (hub index built inside) -> validation -> destroy; and the re-colouring of a
persistent graph beside it.  Usage: tools/step_timing.py [workload] [steps]."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from gcolor_amd.engine import DeviceGraph  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "rmat24"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.cuda.set_device(0)
    t0 = time.time()
    dg0, _ = bench.build_graph(bench.WORKLOADS[wl])
    d_rp, d_col = bench.resident_csr(dg0, torch)
    n, nnz, sym = dg0.n, dg0.nnz, dg0.symmetric
    print(f"{wl}: n={n} nnz={nnz} built in {time.time() - t0:.1f} s", flush=True)
    rec = [dg0.color("A", want_rounds=False, want_colors=False).device_ms for _ in range(3)]
    print(f"recolour (persistent graph) device ms: {[round(x, 1) for x in rec]}", flush=True)
    dg0.close()
    for i in range(steps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        dg = DeviceGraph.from_device(d_rp.data_ptr(), d_col.data_ptr(), n, nnz, symmetric=sym)
        b = time.perf_counter()
        r = dg.color("A", want_rounds=False, want_colors=False)
        c = time.perf_counter()
        unc, conf = dg.validate()
        d = time.perf_counter()
        dg.close()
        e = time.perf_counter()
        print(f"step {i}: total {1e3 * (e - a):.1f} ms = create {1e3 * (b - a):.1f} + colour {1e3 * (c - b):.1f} "
              f"(device {r.device_ms:.1f}) + validate {1e3 * (d - c):.1f} + destroy {1e3 * (e - d):.1f}; "
              f"rounds {r.rounds} colours {r.num_colors} unc {unc} conf {conf}", flush=True)
        assert unc == 0 and conf == 0


if __name__ == "__main__":
    main()
