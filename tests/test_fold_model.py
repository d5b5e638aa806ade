"""Variant B's asynchronous fold protocol (tests/fold_model.py, a model of k_b_async) against
the oracle's variant B: random wave interleavings and stale reads leave every colouring
bit-identical (coloring_optimized.py:120-126, 168-200)."""
import os
import sys

import numpy as np
import pytest

from conftest import REPO, fixture_csr, golden_names, load_golden

sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402
from fold_model import model_color_b  # noqa: E402

GOLD_B = [n for n in golden_names() if "B" in load_golden(n)["variants"]
          and "load_error" not in load_golden(n)["variants"]["B"]["run"] and len(load_golden(n)["graph"]) <= 400]


def _random_directed(n, m, seed):
    rng = np.random.default_rng(seed)
    src = np.sort(rng.integers(0, n, m))
    dst = rng.integers(0, n, m)
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


@pytest.mark.parametrize("name", GOLD_B[:12])
def test_fold_model_golden(name):
    ids, adj, rp, col = fixture_csr(load_golden(name))
    o = oracle.c_color(rp, col, "B")
    for seed in range(2):
        colour, _ = model_color_b(rp, col, seed=seed)
        assert colour == list(o["colors"])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("waves,stale", [(1, 0.0), (3, 0.5), (8, 0.9)])
def test_fold_model_random(seed, waves, stale):
    rp, col = _random_directed(120, 600, 50 + seed)
    o = oracle.c_color(rp, col, "B")
    colour, _ = model_color_b(rp, col, seed=seed, waves=waves, stale=stale)
    assert colour == list(o["colors"])
