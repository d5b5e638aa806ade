"""Perf probe (not a parity check): the same 3-D mesh with its vertices numbered in
diagonal-band order (x+y+z, then file order) against the natural numbering.  The
colourings differ (ties follow positions), the round structure does not: this measures
what a locality-preserving layout is worth to the mesh's rounds."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
from gcolor_amd.engine import DeviceGraph

def mesh_csr(nx, ny, nz, order):
    n = nx * ny * nz
    v = np.arange(n, dtype=np.int64)
    x, y, z = v % nx, (v // nx) % ny, v // (nx * ny)
    if order == "natural":
        perm = v
    else:
        perm = np.argsort(((x + y + z) << 34) | v, kind="stable")  # new -> old
    ipos = np.empty(n, np.int64); ipos[perm] = v                   # old -> new
    del x, y, z
    ox, oy, oz = perm % nx, (perm // nx) % ny, perm // (nx * ny)
    nbr = []
    for cond, d in ((ox > 0, -1), (ox < nx - 1, 1), (oy > 0, -nx), (oy < ny - 1, nx), (oz > 0, -nx * ny), (oz < nz - 1, nx * ny)):
        nbr.append(np.where(cond, ipos[np.clip(perm + d, 0, n - 1)], -1).astype(np.int32))
    del ox, oy, oz
    M = np.stack(nbr, axis=1); del nbr
    deg = (M >= 0).sum(1)
    rp = np.zeros(n + 1, np.int64); np.cumsum(deg, out=rp[1:])
    col = M[M >= 0]
    return rp, col

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 256
for order in ("natural", "diagonal"):
    t = time.time()
    rp, col = mesh_csr(nx, nx, nx, order)
    dg = DeviceGraph.from_csr(rp, col, symmetric=True)
    del col
    bt = time.time() - t
    ts = []
    for i in range(4):
        r = dg.color("A", want_rounds=False, want_colors=False)
        ts.append(r.device_ms)
    print(f"mesh {nx}^3 {order}: build {bt:.1f} s, rounds {r.rounds}, colours {r.max_color + 1}, device ms {[round(x, 1) for x in ts]}", flush=True)
    dg.close()
