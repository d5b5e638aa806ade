#!/usr/bin/env python3
"""GPU box, once: the full-size fixture of R-MAT-27 (the 8-GPU weak-scaling graph, 4.2e9
entries) from the multi-core restatement oracle/gcolor_omp.c (pinned bit-exact to the
single-thread oracle at R-MAT-20 and R-MAT-22, tests/test_oracle_omp.py): the device graph's
identity (sha256 of its row offsets and of its rows sorted by neighbour) and the restatement's
colouring (per-round records, sha256 of the colours and of the round each vertex was coloured
in).  The restatement takes minutes on the box's 16 threads, too long for the GPU suite; its
run is kept as tests/golden/rmat_omp_s27.json and tests/test_gpu_fullsize.py compares the
one-GPU engine against it.  Heartbeat lines every 20 s while it runs.
Usage: python tools/make_rmat27_omp_fixture.py OUT.json [scale]"""
import hashlib
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gcolor_amd.engine import DeviceGraph  # noqa: E402
from oracle import oracle  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = sys.argv[1]
    scale = int(sys.argv[2]) if len(sys.argv) > 2 else 27
    torch.cuda.set_device(0)
    t0 = time.time()
    with DeviceGraph.rmat(scale, 16, seed=1) as dg:
        d_rp, d_col = bench.resident_csr(dg, torch)
    rp = d_rp.cpu().numpy()
    col = d_col.cpu().numpy()
    del d_rp, d_col
    torch.cuda.empty_cache()
    rec = {"generator": f"gc_graph_create_rmat({scale}, 16, 0.57, 0.19, 0.19, seed=1)", "scale": scale,
           "n": int(len(rp) - 1), "nnz": int(len(col)), "rp_sha256": sha(rp), "col_sorted_rows_sha256": sha(col)}
    print(f"R-MAT-{scale}: n={rec['n']} nnz={rec['nnz']} on the host in {time.time() - t0:.0f} s", flush=True)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or 16
    res = {}

    def run():
        res["o"] = oracle.omp_color(rp, col, symmetric=True, threads=threads)

    t0 = time.time()
    th = threading.Thread(target=run)
    th.start()
    while th.is_alive():
        th.join(20)
        print(f"  gcolor_omp.c running, {time.time() - t0:.0f} s", flush=True)
    o = res["o"]
    rec.update({"oracle": f"oracle/gcolor_omp.c ({threads} threads)", "seconds": round(time.time() - t0, 1),
                "status": int(o["status"]), "rounds": int(o["rounds"]), "max_color": int(o["max_color"]),
                "reseeds": int(o["reseeds"]),
                "colors_sha256": sha(o["colors"].astype(np.int32)),
                "colored_round_sha256": sha(o["colored_round"].astype(np.int32)),
                **{"round_" + k: [int(x) for x in o["round_" + k]] for k in ("U", "F", "maxmex", "accepted", "seeds")}})
    with open(out, "w") as f:
        json.dump(rec, f)
    print(f"wrote {out}: {rec['rounds']} rounds, {rec['max_color'] + 1} colours, {rec['seconds']} s", flush=True)


if __name__ == "__main__":
    main()
