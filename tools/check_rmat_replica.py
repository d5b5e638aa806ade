#!/usr/bin/env python3
"""GPU box: the device R-MAT generator (gc_graph_create_rmat) against its numpy replica in
tests/golden/make_rmat_fixtures.py (the full-size parity fixtures are built from the
replica): row offsets and rows sorted by neighbour, equal at the given scales."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"), os.path.join(REPO, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gcolor_amd.engine import DeviceGraph  # noqa: E402
from make_rmat_fixtures import rmat_device_csr  # noqa: E402

torch.cuda.set_device(0)
for s in [int(x) for x in (sys.argv[1:] or ["12", "16", "20"])]:
    with DeviceGraph.rmat(s, 16, seed=1) as dg:
        d_rp, d_col = bench.resident_csr(dg, torch)
    rp, col = d_rp.cpu().numpy(), d_col.cpu().numpy()
    rp2, col2 = rmat_device_csr(s)
    ok = np.array_equal(rp, rp2) and np.array_equal(col[:len(col2)], col2) and len(col) >= len(col2)
    print(f"scale {s}: device n={len(rp) - 1} nnz={rp[-1]}, replica nnz={rp2[-1]}: {'EQUAL' if ok else 'DIFFERENT'}",
          flush=True)
    assert ok
