"""GPU parity of the host round pipeline's launch shortcuts (csrc/gc_engine.hip, Run):

* once 16 rounds ran without a second Jones-Plassmann sweep, rounds are enqueued without
  k_sweep_tail; a later round that needs more sweeps makes k_commit ask the host for them
  (GC_H_SWEEPS) -- here a long path (one-sweep rounds) followed, through an E1 re-seed, by a
  dense random component whose rounds need deep JP chains;
* k_propose_block is not launched when no vertex can be heavy or wide (maxdeg < 64).
Every run must match the oracle bit for bit (colours and per-round records)."""
import os
import random
import sys

import pytest

from test_gpu_parity import _dg, assert_same_run

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _path_then_dense(plen, m, deg, seed, star=150):
    """A star (the seed: the highest degree) at the head of a path, then, disconnected, a
    dense random component that only an E1 re-seed reaches after the path is done."""
    rng = random.Random(seed)
    adj = [[] for _ in range(plen + m + star)]
    for i in range(plen - 1):
        adj[i].append(i + 1)
        adj[i + 1].append(i)
    for leaf in range(plen + m, plen + m + star):
        adj[0].append(leaf)
        adj[leaf].append(0)
    for _ in range(m * deg // 2):
        a, b = rng.randrange(m), rng.randrange(m)
        if a != b:
            adj[plen + a].append(plen + b)
            adj[plen + b].append(plen + a)
    from gcolor_amd.graphio import csr_from_adjacency
    return csr_from_adjacency(adj)


@pytest.mark.parametrize("plen,m,deg,seed", [(120, 400, 10, 1), (300, 2000, 24, 2), (60, 3000, 70, 3)])
def test_tail_skip_then_deep_round(plen, m, deg, seed):
    rp, col = _path_then_dense(plen, m, deg, seed)
    o = oracle.c_color(rp, col, "A")
    assert max(o["round_U"]) > 0
    with _dg().from_csr(rp, col) as dg:
        assert_same_run(dg.color("A"), o)
        top = int(o["max_color"])
        assert_same_run(dg.color("A", num_colors=max(1, top)), oracle.c_color(rp, col, "A", k=max(1, top)))


def test_mesh_like_rounds():
    """A 2-D grid: every round decided by its first sweep; no propose_block launches."""
    w = 40
    adj = [[] for _ in range(w * w)]
    for y in range(w):
        for x in range(w):
            v = y * w + x
            if x + 1 < w:
                adj[v].append(v + 1)
                adj[v + 1].append(v)
            if y + 1 < w:
                adj[v].append(v + w)
                adj[v + w].append(v)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    o = oracle.c_color(rp, col, "A")
    with _dg().from_csr(rp, col) as dg:
        assert_same_run(dg.color("A"), o)


PIPE_SETTINGS = [
    {"GC_FUSE": "0"},                               # a k_propose launch every round
    {"GC_TICKET_CLOSE": "0"},                       # a k_close launch every round
    {"GC_FUSE": "0", "GC_TICKET_CLOSE": "0"},
    {"GC_SNAP_COPY": "1"},                          # copy-engine snapshot of the control block
    {"GC_CLAIM_DIRECT": "1"},                       # fused commit claims with one atomic
    {"GC_BATCH_MAX": "1"},                          # a host wait after every round
]


@pytest.mark.parametrize("env", PIPE_SETTINGS, ids=["nofuse", "noticket", "nofuse_noticket", "snapcopy",
                                                     "claimdirect", "batch1"])
def test_pipeline_settings(monkeypatch, env):
    """The fused commit (next round's proposals made by the commit), the commit that closes
    its round, the pinned snapshot and their switched-off forms all match the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from gcolor_amd.generators import reference_csr
    graphs = [_path_then_dense(120, 400, 10, 1), reference_csr(10000, 8, random.Random(3))]
    w = 30
    adj = [[] for _ in range(w * w)]
    for y in range(w):
        for x in range(w):
            v = y * w + x
            if x + 1 < w:
                adj[v].append(v + 1)
                adj[v + 1].append(v)
            if y + 1 < w:
                adj[v].append(v + w)
                adj[v + w].append(v)
    from gcolor_amd.graphio import csr_from_adjacency
    graphs.append(csr_from_adjacency(adj))
    for rp, col in graphs:
        o = oracle.c_color(rp, col, "A")
        with _dg().from_csr(rp, col) as dg:
            assert_same_run(dg.color("A"), o)
            top = int(o["max_color"])
            for k in sorted({1, max(1, top)}):
                assert_same_run(dg.color("A", num_colors=k), oracle.c_color(rp, col, "A", k=k))
