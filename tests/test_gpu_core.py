"""GPU parity of the hub core (csrc/gc_core.hip) against the CPU oracle.

Once the uncoloured hubs fit the core (GC_CORE_MAX = 8192), k_hub_core decides a round's hub
JP in one workgroup: the hub proposers grouped by candidate in LDS, each class's winners taken
in rank order, a winner's listers struck from a bitset of the core's adjacency.  It restates
resolve_collisions (coloring.py:56-70) for the hubs, so every colouring must equal the oracle's
bit for bit -- and the rounds it cannot take (more winners in a class than GC_HUB_CORE_ITERS,
lights still undecided) fall back to k_sweep_async without a trace in the result.
"""
import os
import sys

import numpy as np
import pytest

from test_gpu_parity import _dg, assert_same_run

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu

CORE_ENV = ("GC_HUB_T", "GC_HUB_CORE", "GC_HUB_CORE_CAP", "GC_HUB_CORE_ITERS", "GC_HUB_CORE_MINF", "GC_ASYNC",
            "GC_ASYNC_BUDGET_US")


@pytest.fixture
def coreenv(monkeypatch):
    for k in CORE_ENV:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GC_HUB_CORE", "1")  # opt-in (measured no faster than the asynchronous JP alone)
    monkeypatch.setenv("GC_HUB_CORE_MINF", "0")  # the core in every round it can take (small graphs)
    return monkeypatch


@pytest.mark.parametrize("scale,hub_t", [(14, "64"), (16, "128"), (12, "0"), (18, "512")])
def test_rmat_core_rounds(coreenv, scale, hub_t):
    """R-MAT graphs whose hub cores are built early: the core decides most rounds (core_rounds
    > 0), and the colouring, every per-round record and the bounded attempts equal the oracle."""
    coreenv.setenv("GC_HUB_T", hub_t)
    with _dg().rmat(scale, 16, seed=scale) as dg:
        rp, col = dg.export()
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert_same_run(g, o)
        assert g.core_rounds > 0 and g.async_aborts == 0
        k = max(1, int(o["max_color"]) // 2)
        assert_same_run(dg.color("A", num_colors=k), oracle.c_color(rp, col, "A", k=k))
        coreenv.setenv("GC_HUB_CORE", "0")  # the default
        off = dg.color("A")
        assert off.core_rounds == 0
        assert_same_run(off, o)


def _wide_class_graph(nhubs=300, leaves=600, path=8):
    """A seed hub S (the argmax of (deg, pos)) starts a path p1..p_path to a light vertex c that
    every one of `nhubs` pairwise non-adjacent hubs lists (each with `leaves` private leaves):
    the round after c is coloured, all of them propose the same candidate and ALL win -- one
    class with `nhubs` winners, after the core was built (and before round 16, when a graph whose
    rounds all ended in their first sweep stops enqueueing the JP's later sweeps)."""
    n0 = 0
    adj = {}

    def add(u, v):
        adj.setdefault(u, []).append(v)
        adj.setdefault(v, []).append(u)

    hubs = list(range(nhubs))
    c = nhubs
    p = list(range(nhubs + 1, nhubs + 1 + path))
    s = nhubs + 1 + path
    nxt = s + 1
    for h in hubs:
        add(h, c)
        for _ in range(leaves):
            add(h, nxt)
            nxt += 1
    add(p[-1], c)
    for a, b in zip(p, p[1:]):
        add(a, b)
    add(s, p[0])
    for _ in range(leaves + 100):  # S's own leaves: it is the seed
        add(s, nxt)
        nxt += 1
    n = nxt
    from gcolor_amd.graphio import csr_from_adjacency
    return csr_from_adjacency([adj.get(v, []) for v in range(n0, n)])


@pytest.mark.parametrize("iters", [None, "5", "4", "1"])
def test_wide_class_falls_back_or_fits(coreenv, iters):
    """One class with 300 winners -- the only round with hub proposers: the core decides it in
    five windows of 64 (default, GC_HUB_CORE_ITERS=5); allowed fewer windows, it hands the round
    to k_sweep_async, which must give the same colouring."""
    if iters:
        coreenv.setenv("GC_HUB_CORE_ITERS", iters)
    rp, col = _wide_class_graph()
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert_same_run(g, o)
        assert g.async_aborts == 0
        assert g.core_rounds == (1 if iters in (None, "5") else 0)


def test_core_with_forced_async_give_up(coreenv):
    """The core's fallback rounds under a zero async budget: k_sweep_async hands them to host
    sweeps -- still the oracle's colouring."""
    coreenv.setenv("GC_HUB_CORE_ITERS", "1")
    coreenv.setenv("GC_ASYNC_BUDGET_US", "0")
    rp, col = _wide_class_graph(nhubs=40, path=6)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        assert_same_run(dg.color("A"), oracle.c_color(rp, col, "A"))
