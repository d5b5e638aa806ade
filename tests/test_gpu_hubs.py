"""GPU parity of the hub path (csrc/gc_hubs.hip) against the CPU oracle.

Hubs keep pushed state instead of re-reading their rows: a forbidden-colour bitmap
(colours of coloured listed neighbours) for assign_color's mex (coloring.py:44-54), and
for resolve_collisions (coloring.py:56-70) a flag raised by light winners of the hub's
candidate, after which the hub's Jones-Plassmann sweeps read only the lower-rank hubs it
lists.  The threshold (GC_HUB_T) and the bitmap width (GC_HUB_W words) are shrunk here so
that small graphs put most vertices on the hub path (hub-hub JP chains, light-only and
hub-only rounds) and reach the row-scan fallback for colours past the bitmap.  Every run must match the oracle bit for
bit: colours, per-round records, the round each vertex was coloured, bounded attempts.
"""
import os
import random
import sys

import numpy as np
import pytest

from test_gpu_parity import _dg, _random_directed, assert_same_run

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu

SETTINGS = [
    {"GC_HUB_T": "0"},                                        # every vertex with a neighbour is a hub
    {"GC_HUB_T": "2"},
    {"GC_HUB_T": "5", "GC_HUB_W": "1"},                       # bitmap of 32 colours: mex fallback
    {"GC_HUB_T": "3"},
    {"GC_HUB_T": "16", "GC_HUB_W": "2"},
    {"GC_HUB_T": "64"},
    {"GC_HUB_T": "512"},                                      # the default
    {"GC_HUB_T": "1024"},
    {"GC_HUB_T": "off"},
    {"GC_HUB_T": "0", "GC_HUB_LONG": "4"},                    # long rows first-read by the whole grid
    {"GC_HUB_T": "2", "GC_HUB_LONG": "0"},                    # ... every row
    {"GC_HUB_T": "0", "GC_HUB_LONG": "0", "GC_HUB_PREP": "off"},  # every row walked by its wave
    {"GC_HUB_T": "0", "GC_HUB_SCAN": "0"},                    # pending-list hub JP (gc_hub_jp_wave)
    {"GC_HUB_T": "2", "GC_HUB_SCAN": "0", "GC_HUB_LONG": "0"},
    {"GC_HUB_T": "0", "GC_TAIL_HMAX_HUB": "0", "GC_ASYNC": "0"},  # no hub in the one-workgroup tail sweeps
    {"GC_HUB_T": "2", "GC_TAIL_HMAX_HUB": "128", "GC_ASYNC": "0"},
    {"GC_HUB_T": "0", "GC_TAIL_HMAX_HUB": "4096", "GC_ASYNC": "0"},  # every hub sweep in the tail once lights converge
    {"GC_HUB_T": "2", "GC_SWEEP_LOOP": "1", "GC_ASYNC": "0"},  # the middle of each JP chain in k_sweep_loop
    {"GC_HUB_T": "off", "GC_SWEEP_LOOP": "1", "GC_LOOP_WG": "8", "GC_ASYNC": "0"},
    {"GC_HUB_T": "0", "GC_ASYNC_BUDGET_US": "0"},             # k_sweep_async gives up at once: spills to host sweeps
    {"GC_HUB_T": "2", "GC_ASYNC_BUDGET_US": "0"},
    {"GC_HUB_T": "off", "GC_ASYNC_BUDGET_US": "0"},
    {"GC_HUB_T": "3", "GC_ASYNC_BPC": "1"},                   # one workgroup per CU
    {"GC_HUB_T": "0", "GC_ASYNC": "0"},                       # round 2's full-grid sweeps + tail
    {"GC_HUB_T": "off", "GC_ASYNC": "0"},
    {"GC_HUB_T": "0", "GC_INLINE_PB": "0"},                   # every round's hubs and wide lights in k_propose_block
    {"GC_HUB_T": "512", "GC_INLINE_PB": "0"},
    {"GC_HUB_T": "1024", "GC_ASYNC": "0"},                    # k_propose<1> with the full-grid sweeps
    {"GC_HUB_T": "2", "GC_HUB_W": "2"},                       # a 64-colour bitmap: inline only while colours are few
    {"GC_HUB_T": "0", "GC_HUB_CORE": "1"},                    # the hub core (opt-in) from frontiers of 1024
    {"GC_HUB_T": "512", "GC_HUB_CORE": "1"},
    {"GC_HUB_T": "0", "GC_HUB_CORE": "1", "GC_HUB_CORE_CAP": "16", "GC_HUB_CORE_MINF": "0"},  # a 16-hub core
    {"GC_HUB_T": "2", "GC_HUB_CORE": "1", "GC_HUB_CORE_CAP": "1", "GC_HUB_CORE_MINF": "0"},
    {"GC_HUB_T": "0", "GC_HUB_CORE": "1", "GC_HUB_CORE_MINF": "0"},  # the core in every round it can take
    {"GC_HUB_T": "64", "GC_HUB_CORE": "1", "GC_HUB_CORE_MINF": "0"},
    {"GC_HUB_T": "0", "GC_HUB_CORE": "1", "GC_HUB_CORE_ITERS": "1", "GC_HUB_CORE_MINF": "0"},  # 2nd window: async
    {"GC_HUB_T": "3", "GC_HUB_CORE": "1", "GC_HUB_CORE_ITERS": "1", "GC_HUB_CORE_MINF": "0",
     "GC_ASYNC_BUDGET_US": "0"},                              # ... which gives up to host sweeps
    {"GC_HUB_T": "0", "GC_ASYNC_WG": "1"},                    # k_sweep_async on 4 waves: hundreds of hubs
    {"GC_HUB_T": "2", "GC_ASYNC_WG": "3"},                    # per wave, in 64-hub batches with ragged ends
]
IDS = ["T0", "T2", "T5w1", "T3", "T16w2", "T64", "T512", "T1024", "off", "T0long4", "T2long0", "T0noprep",
       "T0pend", "T2pend_long0", "T0tail0", "T2tail128", "T0tail4096",
       "T2loop", "offloop8", "T0async_abort", "T2async_abort", "offasync_abort", "T3async_bpc1",
       "T0sync", "offsync", "T0noinl", "T512noinl", "T1024sync", "T2w2", "T0core", "T512core", "T0core16",
       "T2core1", "T0coreall", "T64coreall", "T0coreit1", "T3coreit1_abort", "T0async_wg1", "T2async_wg3"]


@pytest.fixture(params=SETTINGS, ids=IDS)
def hubenv(request, monkeypatch):
    for k in ("GC_HUB_T", "GC_HUB_W", "GC_HUB_LONG", "GC_HUB_PREP", "GC_HUB_SCAN", "GC_TAIL_HMAX_HUB", "GC_SWEEP_LOOP",
              "GC_LOOP_WG", "GC_ASYNC", "GC_ASYNC_BUDGET_US", "GC_ASYNC_BPC", "GC_INLINE_PB", "GC_HUB_CORE",
              "GC_HUB_CORE_CAP", "GC_HUB_CORE_ITERS", "GC_HUB_CORE_MINF", "GC_ASYNC_WG"):
        monkeypatch.delenv(k, raising=False)
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


def _check(rp, col, symmetric=False, bounded=True):
    with _dg().from_csr(rp, col, symmetric=symmetric) as dg:
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert_same_run(g, o)
        if os.environ.get("GC_ASYNC_BUDGET_US") is None:  # k_sweep_async never needs its fallback
            assert g.async_aborts == 0
        assert tuple(dg.validate()) == tuple(oracle.c_validate(rp, col, o["colors"]))
        if bounded:
            top = int(o["max_color"])
            for k in sorted({1, max(1, top // 2), top}):
                assert_same_run(dg.color("A", num_colors=k), oracle.c_color(rp, col, "A", k=k))
        return g


def test_reference_generator_graphs(hubenv):
    from gcolor_amd.generators import reference_csr
    for s in (0, 1, 4):
        rp, col = reference_csr(3000, 8, random.Random(s))
        _check(rp, col, symmetric=True)


@pytest.mark.parametrize("seed", range(3))
def test_directed_multigraphs(hubenv, seed):
    rp, col = _random_directed(2000, 12000, seed)
    _check(rp, col)


@pytest.mark.parametrize("scale", [9, 12])
def test_rmat(hubenv, scale):
    with _dg().rmat(scale, 16, seed=scale + 3) as dg:
        rp, col = dg.export()
    _check(rp, col, symmetric=True, bounded=scale < 12)


def test_clique_and_star(hubenv):
    """A 150-clique (mex up to 149, past a 1-word bitmap) joined to a degree-3000 star."""
    n = 150 + 3000
    adj = [[] for _ in range(n)]
    for i in range(150):
        adj[i] = [j for j in range(150) if j != i]
    for leaf in range(150, n):
        adj[0].append(leaf)
        adj[leaf].append(0)
    for leaf in range(151, n, 5):
        adj[leaf].append(leaf - 1)
        adj[leaf - 1].append(leaf)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    _check(rp, col, bounded=False)


def test_uniform_dense(hubenv):
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(20000, 40, 5)
    _check(rp, col, symmetric=True, bounded=False)


def test_threshold_change_rebuilds(monkeypatch):
    """The same handle re-derives its hubs when the threshold changes between calls."""
    with _dg().rmat(11, 16, seed=2) as dg:
        rp, col = dg.export()
        o = oracle.c_color(rp, col, "A")
        for t in ("64", "4", "off", "0", "64"):
            monkeypatch.setenv("GC_HUB_T", t)
            assert_same_run(dg.color("A"), o)


@pytest.mark.parametrize("bigrow", ["0", "8", "64"])
@pytest.mark.parametrize("hub_t", ["0", "4", "1024"])
def test_commit_big_tiles(monkeypatch, bigrow, hub_t):
    """Winners deferred to k_commit_big (in-rows past GC_BIGROW): with a tiny threshold
    hundreds of hub winners per round go through its flat walk, several 256-winner tiles."""
    monkeypatch.setenv("GC_HUB_T", hub_t)
    monkeypatch.setenv("GC_BIGROW", bigrow)
    with _dg().rmat(12, 16, seed=7) as dg:
        rp, col = dg.export()
    _check(rp, col, symmetric=True, bounded=False)
    rp, col = _random_directed(3000, 30000, 11)
    _check(rp, col)


@pytest.mark.parametrize("hub_t", ["512", "95", "100", "1"])
def test_partition_hub_flags_match_gathered_bits(monkeypatch, hub_t):
    """The rank partition marks hub entries from the byte key it gathers anyway (gc_prep.hip,
    round 5; deg gathered only in the key's bucket when it straddles the threshold: 512 and
    100 straddle, 95 does not) and the hub transpose streams those flags; GC_HUB_FLAGS=0 gathers
    a hub bit per entry as before.  Both give the oracle's colouring, round for round -- on an
    R-MAT graph whose hub rows are split into partition segments (rows > 1024 entries)."""
    from gcolor_amd.engine import DeviceGraph
    monkeypatch.setenv("GC_HUB_T", hub_t)
    with DeviceGraph.rmat(16, 16, seed=7) as dg:
        rp, col = dg.export()
    assert np.diff(rp).max() > 2048
    o = oracle.c_color(rp, col, "A")
    for flags in ("1", "0"):
        monkeypatch.setenv("GC_HUB_FLAGS", flags)
        with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
            g = dg.color("A")
            assert g.hubs > 0
            assert_same_run(g, o)
            assert dg.validate() == (0, 0)


def test_inline_proposal_overrun_falls_back(monkeypatch):
    """Hubs proposed inside k_propose<1> need their bitmaps to cover every colour the enqueued
    rounds can reach (the host keeps a margin over the last snapshot's max colour).  With the
    margin forced negative (GC_TEST_INL_MARGIN) and 1-word bitmaps (32 colours), the device
    reports the overrun and the colouring is run again without the inlined proposals
    (no hard error) -- the oracle's colouring, round for round."""
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(12, 16, seed=3) as dg:
        rp, col = dg.export()
    o = oracle.c_color(rp, col, "A")
    assert o["max_color"] > 40
    monkeypatch.setenv("GC_HUB_T", "8")
    monkeypatch.setenv("GC_HUB_W", "1")
    monkeypatch.setenv("GC_TEST_INL_MARGIN", "-1000")
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        assert_same_run(dg.color("A"), o)
