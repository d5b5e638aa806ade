"""GPU parity of the seeded-priority rounds and the speculative first-fit mode
(csrc/gc_priority.hip) against the oracle's restatement of the same semantics
(oracle_color_prio, itself cross-checked against a pure-Python restatement in
tests/test_oracle_priority.py).  Bit-exact: colours, per-round records, the round each
vertex was coloured, bounded attempts.  Switching the rank re-partitions the rows in
place; the reference path must still match the oracle afterwards.
"""
import os
import random
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden
from test_gpu_parity import _dg, _random_directed, assert_same_run

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu

MODES = [(7, False), (7, True), (None, True), (2**40 + 3, False)]
MIDS = ["seed7", "seed7spec", "refspec", "seedbig"]
GOLD = [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]]


def _o(rp, col, seed, spec, k=None):
    return oracle.c_color_prio(rp, col, k=k, priority=0 if seed is None else 1, seed=seed or 0, speculative=spec)


def _check(dg, rp, col, seed, spec, bounded=True):
    o = _o(rp, col, seed, spec)
    g = dg.color("A", priority=seed, speculative=spec)
    assert_same_run(g, o)
    if bounded:
        top = int(o["max_color"])
        for k in sorted({0, 1, max(1, top // 2), top}):
            assert_same_run(dg.color("A", num_colors=k, priority=seed, speculative=spec), _o(rp, col, seed, spec, k))
    return g


@pytest.mark.parametrize("mode", MODES, ids=MIDS)
@pytest.mark.parametrize("name", GOLD)
def test_golden_graphs(name, mode):
    _, _, rp, col = fixture_csr(load_golden(name))
    with _dg().from_csr(rp, col) as dg:
        _check(dg, rp, col, *mode)
        assert_same_run(dg.color("A"), oracle.c_color(rp, col, "A"))  # back to (deg, pos)


@pytest.mark.parametrize("mode", MODES, ids=MIDS)
def test_random_graphs(mode):
    from gcolor_amd.engine import uniform_csr
    from gcolor_amd.generators import reference_csr
    rp, col = reference_csr(10000, 8, random.Random(1))  # stray components: E1 in the seeded JP mode
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        _check(dg, rp, col, *mode)
    rp, col = _random_directed(3000, 12000, 4)
    with _dg().from_csr(rp, col) as dg:
        _check(dg, rp, col, *mode)
    rp, col = uniform_csr(200_000, 16, 5)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        g = _check(dg, rp, col, *mode, bounded=False)
        assert dg.validate() == (0, 0)
        assert g.max_color < 17


@pytest.mark.parametrize("mode", MODES, ids=MIDS)
def test_rmat_and_mesh(mode):
    DG = _dg()
    with DG.rmat(12, 16, seed=5) as dg:
        rp, col = dg.export()
        _check(dg, rp, col, *mode, bounded=False)
        assert dg.validate() == (0, 0)
        a = dg.color("A")  # the hub engine after a re-partition
        assert_same_run(a, oracle.c_color(*dg.export(), "A"))
    with DG.mesh(12, 10, 8) as dg:
        rp, col = dg.export()
        _check(dg, rp, col, *mode, bounded=False)


def test_colour_counts_against_reference():
    """The north star's "no more colours than the reference" for the fast modes is
    reported per graph: here only validity is required."""
    from gcolor_amd.generators import reference_csr
    for s in range(3):
        rp, col = reference_csr(10000, 8, random.Random(s))
        with _dg().from_csr(rp, col, symmetric=True) as dg:
            ref = dg.color("A").max_color + 1
            for seed, spec in MODES:
                g = dg.color("A", priority=seed, speculative=spec)
                assert g.ok and dg.validate() == (0, 0)
                assert g.max_color + 1 <= ref + 2


@pytest.mark.parametrize("hub_t,hub_w", [("0", "128"), ("64", "1"), ("off", "128")])
@pytest.mark.parametrize("mode", MODES[:3], ids=MIDS[:3])
def test_modes_with_hub_bitmaps(monkeypatch, hub_t, hub_w, mode):
    """Seeded and speculative rounds propose hubs from pushed forbidden-colour bitmaps (no
    hub JP): every threshold, a one-word bitmap (row-scan fallback past 32 colours) and
    hubs off agree with the oracle; the reference path after them too (hub lists rebuilt
    for the (deg, pos) partition)."""
    monkeypatch.setenv("GC_HUB_T", hub_t)
    monkeypatch.setenv("GC_HUB_W", hub_w)
    with _dg().rmat(12, 16, seed=7) as dg:
        rp, col = dg.export()
        _check(dg, rp, col, *mode, bounded=False)
        assert_same_run(dg.color("A"), oracle.c_color(*dg.export(), "A"))
    n = 40 + 3000
    adj = [[] for _ in range(n)]
    for i in range(40):  # a clique of hubs (colours past a 1-word bitmap), each with leaves
        adj[i] += [j for j in range(40) if j != i]
    for leaf in range(40, n):
        adj[leaf % 40].append(leaf)
        adj[leaf].append(leaf % 40)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    with _dg().from_csr(rp, col) as dg:
        _check(dg, rp, col, *mode)
