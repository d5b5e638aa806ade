#!/usr/bin/env python3
"""Full-size parity fixtures for the R-MAT configurations.

The single-thread C oracle (oracle/gcolor_oracle.c, pinned to the reference's own golden
vectors by tests/test_oracle_golden.py) is far too slow to run inside the GPU suite at C3's
size (R-MAT-24: ~20 min per variant on one core).  This script runs it ONCE, here, and keeps
what a test needs to compare a full colouring exactly:

  * the graph: a numpy replica of the device generator (gc_graph_create_rmat, k_rmat_edges in
    csrc/gc_graph.hip: a counter-based splitmix64 stream per edge, so the graph is a pure
    function of (scale, edge factor, a, b, c, seed)), symmetrised, de-duplicated, self-loops
    dropped; sha256 of its row offsets and of its rows sorted by neighbour -- the GPU test
    checks the device graph against these first;
  * per variant (A = coloring.py, B = coloring_optimized.py): status, rounds, every per-round
    record (U, F, max mex, accepted, seeds), max colour, and sha256 of the colour array and of
    the round each vertex was coloured in.

Output: tests/golden/rmat_oracle_s<scale>.json.  Usage:
  python tests/golden/make_rmat_fixtures.py 24 A B     (C3, both variants: ~40 min)
  python tests/golden/make_rmat_fixtures.py pin22      (the CPU pin of gcolor_omp.c: the oracle
                                                       on tests/test_oracle_omp.py's R-MAT-22)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix(x):
    """splitmix64 finaliser (gc_splitmix, csrc/gc_graph.hip) on a uint64 array (wrapping)."""
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def rmat_device_csr(scale, ef=16, a=0.57, b=0.19, c=0.19, seed=1, chunk=1 << 24):
    """The exact CSR gc_graph_create_rmat builds (rows sorted by neighbour)."""
    n = 1 << scale
    m = ef * n
    ta = np.uint64(int(a * 4294967296.0))
    tb = np.uint64(int((a + b) * 4294967296.0))
    tc = np.uint64(int((a + b + c) * 4294967296.0))
    sc = np.uint64(scale)
    keys = []
    with np.errstate(over="ignore"):
        for i0 in range(0, m, chunk):
            i = np.arange(i0, min(m, i0 + chunk), dtype=np.uint64)
            src = np.zeros(i.shape, np.uint64)
            dst = np.zeros(i.shape, np.uint64)
            h = None
            for lvl in range(scale):
                if lvl % 2 == 0:
                    h = splitmix(np.uint64(seed) ^ splitmix(i * np.uint64(64) + np.uint64(lvl >> 1)))
                r = (h >> np.uint64(32)) if lvl % 2 else (h & np.uint64(0xFFFFFFFF))
                q = np.where(r < ta, 0, np.where(r < tb, 1, np.where(r < tc, 2, 3))).astype(np.uint64)
                src = (src << np.uint64(1)) | (q >> np.uint64(1))
                dst = (dst << np.uint64(1)) | (q & np.uint64(1))
            keep = src != dst
            src, dst = src[keep], dst[keep]
            keys.append((src << sc) | dst)
            keys.append((dst << sc) | src)
    k = np.unique(np.concatenate(keys))
    del keys
    col = (k & np.uint64(n - 1)).astype(np.int32)
    rows = (k >> sc).astype(np.int64)
    del k
    rp = np.searchsorted(rows, np.arange(n + 1, dtype=np.int64), side="left").astype(np.int64)
    return rp, col


def rmat_device_csr_lowmem(scale, ef=16, a=0.57, b=0.19, c=0.19, seed=1, chunk=1 << 24):
    """rmat_device_csr with a bounded peak (R-MAT-26 in ~30 GB instead of ~70): the keys go
    into one preallocated array, sorted in place and de-duplicated by a forward chunked
    compaction; the row offsets are searched on the keys directly.  Same CSR, bit for bit
    (tests/test_host.py::test_rmat_lowmem_matches compares the two at small scales)."""
    n = 1 << scale
    m = ef * n
    ta = np.uint64(int(a * 4294967296.0))
    tb = np.uint64(int((a + b) * 4294967296.0))
    tc = np.uint64(int((a + b + c) * 4294967296.0))
    sc = np.uint64(scale)
    k = np.empty(2 * m, np.uint64)
    w = 0
    with np.errstate(over="ignore"):
        for i0 in range(0, m, chunk):
            i = np.arange(i0, min(m, i0 + chunk), dtype=np.uint64)
            src = np.zeros(i.shape, np.uint64)
            dst = np.zeros(i.shape, np.uint64)
            h = None
            for lvl in range(scale):
                if lvl % 2 == 0:
                    h = splitmix(np.uint64(seed) ^ splitmix(i * np.uint64(64) + np.uint64(lvl >> 1)))
                r = (h >> np.uint64(32)) if lvl % 2 else (h & np.uint64(0xFFFFFFFF))
                q = np.where(r < ta, 0, np.where(r < tb, 1, np.where(r < tc, 2, 3))).astype(np.uint64)
                src = (src << np.uint64(1)) | (q >> np.uint64(1))
                dst = (dst << np.uint64(1)) | (q & np.uint64(1))
            keep = src != dst
            src, dst = src[keep], dst[keep]
            cnt = len(src)
            k[w:w + cnt] = (src << sc) | dst
            k[w + cnt:w + 2 * cnt] = (dst << sc) | src
            w += 2 * cnt
    k = k[:w]
    k.sort()
    u = 0
    prev = None
    for i0 in range(0, w, chunk):
        blk = k[i0:i0 + chunk].copy()  # read before any of it is overwritten (u <= i0)
        keep = np.empty(len(blk), bool)
        keep[1:] = blk[1:] != blk[:-1]
        keep[0] = prev is None or blk[0] != prev
        prev = blk[-1]
        blk = blk[keep]
        k[u:u + len(blk)] = blk
        u += len(blk)
    k = k[:u]
    col = np.empty(u, np.int32)
    for i0 in range(0, u, chunk):
        col[i0:i0 + chunk] = (k[i0:i0 + chunk] & np.uint64(n - 1)).astype(np.int32)
    rp = np.searchsorted(k, np.arange(n + 1, dtype=np.uint64) << sc, side="left").astype(np.int64)
    return rp, col


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pin_fixture(scale):
    """The single-thread oracle's variant-A run on tests/test_oracle_omp.py's numpy R-MAT graph
    (rmat_csr(scale, 16, seed=scale)): the pin of the multi-core restatement gcolor_omp.c at a
    size where the oracle takes minutes (tests/test_oracle_omp.py::test_rmat_pinned_fixture)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle import oracle
    from test_oracle_omp import rmat_csr
    rp, col = rmat_csr(scale, 16, seed=scale)
    t0 = time.time()
    o = oracle.c_color(rp, col, "A", max_rounds=1 << 14)
    rec = {"generator": f"tests/test_oracle_omp.py rmat_csr({scale}, 16, seed={scale})", "scale": scale,
           "n": int(len(rp) - 1), "nnz": int(len(col)), "rp_sha256": sha(rp), "col_sha256": sha(col),
           "oracle": "oracle/gcolor_oracle.c (one thread)", "seconds": round(time.time() - t0, 1),
           "status": int(o["status"]), "rounds": int(o["rounds"]), "max_color": int(o["max_color"]),
           "colors_sha256": sha(o["colors"].astype(np.int32)),
           "colored_round_sha256": sha(o["colored_round"].astype(np.int32)),
           **{"round_" + k: [int(x) for x in o["round_" + k]] for k in ("U", "F", "maxmex", "accepted", "seeds")}}
    out_path = os.path.join(HERE, f"rmat_csr_oracle_s{scale}.json")
    with open(out_path, "w") as f:
        json.dump(rec, f)
    print("wrote", out_path, rec["rounds"], "rounds", rec["seconds"], "s")


def main():
    if len(sys.argv) > 1 and sys.argv[1].startswith("pin"):
        return pin_fixture(int(sys.argv[1][3:]))
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    variants = sys.argv[2:] or ["A", "B"]
    from oracle import oracle
    t0 = time.time()
    # scales >= 26: the low-memory generator, and the CSR cached as .npy (GC_FIXTURE_CACHE, default
    # /tmp) so that variants can run as separate processes over one memory-mapped graph
    cache = os.environ.get("GC_FIXTURE_CACHE", "/tmp")
    rp_p, col_p = (os.path.join(cache, f"rmat_s{scale}_{x}.npy") for x in ("rp", "col"))
    if scale >= 26 and os.path.exists(rp_p) and os.path.exists(col_p):
        rp, col = np.load(rp_p, mmap_mode="r"), np.load(col_p, mmap_mode="r")
    elif scale >= 26:
        rp, col = rmat_device_csr_lowmem(scale)
        np.save(rp_p, rp)
        np.save(col_p, col)
    else:
        rp, col = rmat_device_csr(scale)
    print(f"R-MAT-{scale}: n={len(rp) - 1} nnz={len(col)} generated in {time.time() - t0:.0f} s", flush=True)
    if "gen" in variants:
        return
    out_path = os.path.join(HERE, f"rmat_oracle_s{scale}.json")
    graph = {"generator": "gc_graph_create_rmat(scale, 16, 0.57, 0.19, 0.19, seed=1), numpy replica",
             "scale": scale, "n": int(len(rp) - 1), "nnz": int(len(col)),
             "rp_sha256": sha(rp), "col_sorted_rows_sha256": sha(col)}
    for v in variants:
        t0 = time.time()
        o = oracle.c_color(rp, col, v, max_rounds=1 << 14)
        dt = time.time() - t0
        res = {
            "oracle": "oracle/gcolor_oracle.c (one thread)", "seconds": round(dt, 1),
            "status": int(o["status"]), "rounds": int(o["rounds"]), "max_color": int(o["max_color"]),
            "colors_sha256": sha(o["colors"].astype(np.int32)),
            "colored_round_sha256": sha(o["colored_round"].astype(np.int32)),
            **{"round_" + k: [int(x) for x in o["round_" + k]] for k in ("U", "F", "maxmex", "accepted", "seeds")}}
        print(f"variant {v}: {o['rounds']} rounds, {o['max_color'] + 1} colours, {dt:.0f} s", flush=True)
        import fcntl  # variants may run as concurrent processes: read-update-write under a lock
        with open(out_path + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            rec = json.load(open(out_path)) if os.path.exists(out_path) else {}
            rec.update(graph)
            rec.setdefault("variants", {})[v] = res
            with open(out_path, "w") as f:
                json.dump(rec, f)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
