"""The identity behind gc_validate's low-part count for symmetric graphs (csrc/gc_prep.hip,
k_validate_tiles HALF), checked on the CPU with numpy.

coloring.py:149-162 counts conflicts per listed entry (v, u): colour[u] == colour[v], duplicates
and self-loops included, uncoloured (-1) pairs too.  In a symmetric list every entry (v, u) with
u != v has a mirror (u, v) of the same multiplicity, and the rank partition (deg, pos) puts
exactly one of the two in a low part (a strict order), never a self-loop.  So the directed
count equals 2 x the low parts' conflicts + the self-loop entries.
"""
import numpy as np
import pytest


def _sym_multigraph(rng, n, m, loops):
    a = rng.integers(0, n, m)
    b = rng.integers(0, n, m)
    a = np.concatenate([a, a[: m // 10]])  # duplicates
    b = np.concatenate([b, b[: m // 10]])
    keep = a != b
    s = np.concatenate([a[keep], b[keep], rng.integers(0, n, loops)])
    d = np.concatenate([b[keep], a[keep], np.zeros(0, np.int64)])
    d = np.concatenate([d, s[len(d):]])  # the self-loops: one entry each
    return s, d


@pytest.mark.parametrize("seed", range(6))
def test_directed_count_is_twice_low_plus_selfloops(seed):
    rng = np.random.default_rng(seed)
    n = 300
    src, dst = _sym_multigraph(rng, n, 2000, 25)
    deg = np.bincount(src, minlength=n)
    # rank(u) < rank(v) iff (deg, pos) lexicographically smaller (coloring.py:64 tie-break on id)
    low = (deg[dst] < deg[src]) | ((deg[dst] == deg[src]) & (dst < src))
    for palette in (2, 5, 300):
        colors = rng.integers(-1, palette, n)
        same = colors[src] == colors[dst]
        directed = int(same.sum())
        assert directed == 2 * int((same & low).sum()) + int((src == dst).sum())
        assert not (low & (src == dst)).any()
