"""The asynchronous JP protocol (tests/jp_model.py, a model of k_sweep_async's light passes)
against the oracle's variant A: random wave interleavings and stale state reads leave every
colouring and every round record bit-identical (coloring.py:56-70, 73-132)."""
import sys

import numpy as np
import pytest

from conftest import REPO, fixture_csr, golden_names, load_golden

sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402
from jp_model import model_color_a  # noqa: E402

GOLD = [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]
        and len(load_golden(n)["graph"]) <= 400]


def _random_directed(n, m, seed):
    rng = np.random.default_rng(seed)
    src = np.sort(rng.integers(0, n, m))
    dst = rng.integers(0, n, m)
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


def _same(rp, col, **kw):
    o = oracle.c_color(rp, col, "A")
    colour, recs = model_color_a(rp, col, **kw)
    assert colour == list(o["colors"])
    assert [r[0] for r in recs] == list(o["round_U"])
    assert [r[1] for r in recs] == list(o["round_F"])
    assert [r[2] for r in recs] == list(o["round_accepted"])
    assert [r[3] for r in recs] == list(o["round_seeds"])


@pytest.mark.parametrize("name", GOLD[:12])
def test_jp_model_golden(name):
    ids, adj, rp, col = fixture_csr(load_golden(name))
    for seed in range(2):
        _same(rp, col, seed=seed)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("waves,stale", [(1, 0.0), (3, 0.5), (8, 0.9)])
def test_jp_model_random(seed, waves, stale):
    """Directed multigraphs with self-loops and stray components (E1 re-seeds)."""
    rp, col = _random_directed(150, 700, 80 + seed)
    _same(rp, col, seed=seed, waves=waves, stale=stale)


@pytest.mark.parametrize("seed", range(3))
def test_jp_model_dense_conflicts(seed):
    """Few candidates, long same-candidate chains: the deepest JP chains per round."""
    rp, col = _random_directed(80, 1600, 200 + seed)
    _same(rp, col, seed=seed, waves=6, stale=0.8)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("hub_t", [0, 4, 9])
def test_jp_model_hub_jp(seed, hub_t):
    """The hub JP: lights first, light winners kill the hubs listing them that propose their
    colour, then the hubs resolve among themselves -- under stale reads, against the oracle."""
    rp, col = _random_directed(150, 900, 300 + seed)
    _same(rp, col, seed=seed, waves=5, stale=0.6, hub_t=hub_t)
