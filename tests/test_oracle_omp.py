"""The multi-core CPU baseline (oracle/gcolor_omp.c) is bench.py's cpu_baseline leg: it
must compute exactly what the single-thread oracle computes (variant A, coloring.py:73-132
+ E1) -- colours and every per-round record -- on the golden set and on graphs with hubs
(deg > 512: its pushed-bitmap / hub-JP path), self-loops, duplicates and asymmetric rows.
No GPU needed."""
import os
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

KEYS = ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds")


def _same(rp, col, symmetric, threads=4):
    c = oracle.c_color(rp, col, "A")
    o = oracle.omp_color(rp, col, symmetric=symmetric, threads=threads)
    assert c["status"] == o["status"] == 0
    assert np.array_equal(c["colors"], o["colors"])
    assert np.array_equal(c["colored_round"], o["colored_round"])
    for k in KEYS:
        assert np.array_equal(c[k], o[k]), k
    assert c["reseeds"] == o["reseeds"]
    return c


def _is_sym(rp, col):
    n = len(rp) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    a = np.unique(src * n + col)
    b = np.unique(col.astype(np.int64) * n + src)
    return a.shape == b.shape and bool(np.array_equal(a, b))


@pytest.mark.parametrize("name", golden_names())
def test_golden_graphs(name):
    rec = load_golden(name)
    if "A" not in rec["variants"] or "load_error" in rec["variants"]["A"]["run"] or not rec["graph"]:
        pytest.skip("no variant-A graph")
    _, _, rp, col = fixture_csr(rec)
    _same(rp, col, _is_sym(rp, col))


def rmat_csr(scale, ef, seed, sym=True):
    """numpy R-MAT (0.57, 0.19, 0.19), self-loops dropped, de-duplicated (test inputs)."""
    rng = np.random.default_rng(seed)
    m = ef << scale
    src = np.zeros(m, np.int64)
    dst = np.zeros(m, np.int64)
    for _ in range(scale):
        r = rng.random(m)
        b_src = r >= 0.57 + 0.19
        b_dst = ((r >= 0.57) & (r < 0.76)) | (r >= 0.95)
        src = 2 * src + b_src
        dst = 2 * dst + b_dst
    keep = src != dst
    src, dst = src[keep], dst[keep]
    if sym:
        src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
    n = 1 << scale
    key = np.unique(src * n + dst)
    src, dst = key // n, key % n
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


@pytest.mark.parametrize("scale,threads", [(12, 1), (14, 4), (15, 8), (16, 8), (18, 8), (20, 8)])
def test_rmat_hubs(scale, threads):
    """R-MAT-16/18 (hubs of 10^4 entries, 157/240 rounds): the restatement the GPU is checked
    against at C3/C4 sizes is pinned to the single-thread oracle where real hubs exist."""
    rp, col = rmat_csr(scale, 16, seed=scale)
    assert np.diff(rp).max() > 512  # the hub path runs
    c = _same(rp, col, True, threads)
    assert oracle.c_validate(rp, col, c["colors"]) == (0, 0)


def test_asymmetric_multigraph():
    rng = np.random.default_rng(5)
    n = 3000
    deg = rng.integers(0, 12, n)
    deg[:3] = 900  # hubs with asymmetric rows
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = rng.integers(0, n, rp[-1]).astype(np.int32)  # duplicates and self-loops included
    _same(rp, col, False)


def test_uniform_generator():
    from gcolor_amd.generators import reference_csr
    import random
    rp, col = reference_csr(10000, 8, random.Random(1))  # random.seed(1): stray components (E1)
    c = _same(rp, col, True)
    assert c["reseeds"] > 0


PIN22 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_csr_oracle_s22.json")


@pytest.mark.skipif(not os.path.exists(PIN22), reason="tests/golden/rmat_csr_oracle_s22.json not generated")
def test_rmat22_pinned_to_oracle_fixture():
    """R-MAT-22 (4.2M vertices, 1.3e8 entries, hubs of 10^5): the restatement the GPU's full-size
    runs are checked against (R-MAT-26/27, C4) pinned to the single-thread oracle where the
    oracle takes minutes -- its run is the committed fixture (tests/golden/make_rmat_fixtures.py
    pin22): the graph (sha256), every per-round record, the colours and the round each vertex
    was coloured in (sha256)."""
    import hashlib
    import json
    fx = json.load(open(PIN22))

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    rp, col = rmat_csr(22, 16, seed=22)
    assert sha(rp) == fx["rp_sha256"] and sha(col) == fx["col_sha256"]
    o = oracle.omp_color(rp, col, symmetric=True, threads=8)
    assert (o["status"], o["rounds"], o["max_color"]) == (fx["status"], fx["rounds"], fx["max_color"])
    for k in KEYS:
        assert [int(x) for x in o[k]] == fx[k], k
    assert sha(o["colors"].astype(np.int32)) == fx["colors_sha256"]
    assert sha(o["colored_round"].astype(np.int32)) == fx["colored_round_sha256"]
