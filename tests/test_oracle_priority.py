"""Seeded priorities and the speculative mode in the oracle (no GPU).

The reference has no seeded-priority mode (its tie-break is (deg, pos), coloring.py:64),
so these semantics are parity-unpinned by the reference's own outputs.  They are pinned by
two independent restatements instead -- the C oracle (oracle_color_prio) and the
pure-Python py_color(priority_seed=..., speculative=...) -- plus identities: priority 0
without speculation IS the reference path, every colouring is valid on symmetric graphs.
"""
import os
import random
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

NAMES = [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]]
SMALL = [n for n in NAMES if len(load_golden(n)["graph"] or []) <= 1000]


def test_hash_matches_python():
    for seed in (0, 1, 42, 2**63 + 5):
        for v in (0, 1, 7, 10**6, 2**31 - 1):
            assert oracle.prio_hash(seed, v) == oracle.py_prio_hash(seed, v)


@pytest.mark.parametrize("name", NAMES)
def test_priority_ref_is_the_reference_path(name):
    _, _, rp, col = fixture_csr(load_golden(name))
    a = oracle.c_color(rp, col, "A")
    b = oracle.c_color_prio(rp, col, priority=0, seed=123)
    assert np.array_equal(a["colors"], b["colors"]) and np.array_equal(a["round_U"], b["round_U"])


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("mode", [(1, False), (1, True), (0, True)])
def test_c_matches_python_restatement(name, mode):
    prio, spec = mode
    _, adj, rp, col = fixture_csr(load_golden(name))
    for seed in (3, 99):
        c = oracle.c_color_prio(rp, col, priority=prio, seed=seed, speculative=spec)
        p = oracle.py_color(adj, "A", priority_seed=seed if prio else None, speculative=spec)
        assert list(c["colors"]) == p["colors"]
        assert list(c["round_U"]) == p["round_U"] and list(c["round_F"]) == p["round_F"]
        assert c["reseeds"] == p["reseeds"]
        top = int(c["max_color"])
        for k in sorted({0, 1, max(1, top // 2), top}):
            ck = oracle.c_color_prio(rp, col, k=k, priority=prio, seed=seed, speculative=spec)
            pk = oracle.py_color(adj, "A", k=k, priority_seed=seed if prio else None, speculative=spec)
            assert ck["status"] == pk["status"] and list(ck["colors"]) == pk["colors"]


def test_seeded_and_speculative_colourings_are_valid():
    from gcolor_amd.generators import reference_csr
    for s in range(4):
        rp, col = reference_csr(5000, 8, random.Random(s))
        for prio, spec in [(1, False), (1, True), (0, True)]:
            o = oracle.c_color_prio(rp, col, priority=prio, seed=s, speculative=spec)
            assert o["status"] == 0 and oracle.c_validate(rp, col, o["colors"]) == (0, 0)
