"""Pin the CPU oracle (C and pure-Python restatements) to the reference's own outputs.

The golden vectors were recorded by tests/golden/make_golden.py, which executed the
reference's unmodified coloring.py / coloring_optimized.py. These tests need no GPU.
"""
import os
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from kloop_emulation import emulate  # noqa: E402

NAMES = golden_names()
CASES = [(n, v) for n in NAMES for v in load_golden(n)["variants"]]


def _symmetric(adj):
    s = set((v, u) for v, a in enumerate(adj) for u in a)
    return all((u, v) in s for v, u in s)


@pytest.mark.parametrize("name,variant", CASES)
def test_unbounded_run_matches_reference(name, variant):
    rec = load_golden(name)
    run = rec["variants"][variant]["run"]
    if "load_error" in run:
        pytest.skip("graph does not load in the reference (CLI-level case)")
    ids, adj, rp, col = fixture_csr(rec)
    c = oracle.c_color(rp, col, variant)
    if run.get("exception"):
        # the reference crashes on an edgeless graph (empty reduce);
        # the restatement colours every isolated vertex 0 instead.
        assert "empty" in run["exception"]
        assert all(len(a) == 0 for a in adj)
        assert (c["colors"] == 0).all()
        return
    if run["hang"]:
        # reference spins at the first zero-proposer round. Without E1 the
        # oracle stops there with the same state; with E1 it completes.
        s = oracle.c_color(rp, col, variant, e1=False)
        assert s["status"] == oracle.STALLED
        ref_u = [u for i, u in enumerate(run["rounds_U"]) if i == 0 or u != run["rounds_U"][i - 1]]
        assert list(s["round_U"]) == ref_u
        got_colored = [r != -1 for r in s["colored_round"]]
        assert got_colored == [r != -1 for r in run["colored_round"]]
        assert c["status"] == oracle.OK and c["reseeds"] > 0
        if _symmetric(adj):
            selfloops = sum(1 for v, a in enumerate(adj) for u in a if u == v)
            assert oracle.c_validate(rp, col, c["colors"]) == (0, selfloops)
        return
    assert run["ok"]
    assert c["status"] == oracle.OK
    assert list(c["colors"]) == run["colors"]
    assert list(c["round_U"]) == run["rounds_U"]
    assert list(c["colored_round"]) == run["colored_round"]
    assert c["reseeds"] == 0


@pytest.mark.parametrize("name,variant", [cv for cv in CASES if len(load_golden(cv[0])["graph"] or []) <= 1000])
def test_python_restatement_matches_c(name, variant):
    rec = load_golden(name)
    if "load_error" in rec["variants"][variant]["run"]:
        pytest.skip("load error case")
    ids, adj, rp, col = fixture_csr(rec)
    c = oracle.c_color(rp, col, variant)
    p = oracle.py_color(adj, variant)
    assert p["status"] == c["status"]
    assert p["colors"] == list(c["colors"])
    assert p["round_U"] == list(c["round_U"])
    assert p["round_F"] == list(c["round_F"])
    assert p["round_maxmex"] == list(c["round_maxmex"])
    assert p["colored_round"] == list(c["colored_round"])
    assert p["reseeds"] == c["reseeds"]
    for k in range(0, int(c["max_color"]) + 2):
        cb = oracle.c_color(rp, col, variant, k=k)
        pb = oracle.py_color(adj, variant, k=k)
        assert (pb["status"], pb["fail_round"], pb["fail_count"]) == (cb["status"], cb["fail_round"], cb["fail_count"])
        assert pb["colors"] == list(cb["colors"])
    assert oracle.py_validate(adj, p["colors"]) == oracle.c_validate(rp, col, c["colors"])


@pytest.mark.parametrize("name,variant", CASES)
def test_cli_kloop_matches_reference(name, variant):
    """The literal k-loop over the oracle reproduces the reference CLI transcript and
    output file (coloring.py:211-241) on every terminating case."""
    rec = load_golden(name)
    cli = rec["variants"][variant]["cli"]
    if cli["hang"] or cli.get("exception") or cli["exit"] != 0:
        pytest.skip("reference CLI does not terminate normally here (Q1/Q4/load error)")
    ids, adj, rp, col = fixture_csr(rec)
    argv = cli["argv"]
    maxdeg_arg = int(argv[argv.index("--max-degree") + 1]) if "--max-degree" in argv else None
    K0 = maxdeg_arg + 1 if maxdeg_arg else max(len(a) for a in adj) + 1
    lines, out = emulate(lambda k: oracle.c_color(rp, col, variant, k=k),
                         lambda colors: oracle.c_validate(rp, col, colors), K0)
    assert lines == cli["stdout"]
    assert cli["output_ids"] == ids
    assert out == cli["output_colors"]


def test_shipped_colors_json_is_variant_b_snapshot():
    """colors.json in the reference == variant B's failed k=2 snapshot."""
    rec = load_golden("graph_json")
    assert rec["variants"]["B"]["cli"]["output_colors"] == [0, 0, 1, -1, 1, -1, 0, 1, 1, 1]
    ids, adj, rp, col = fixture_csr(rec)
    snap = oracle.c_color(rp, col, "B", k=2)
    assert snap["status"] == oracle.FAILED
    assert list(snap["colors"]) == [0, 0, 1, -1, 1, -1, 0, 1, 1, 1]


def test_survey_pins_seed0_10000():
    """Known-answer pins from SURVEY.md §8a (random.seed(0); Graph(10000, 8))."""
    import hashlib
    import json as _json
    rec = load_golden("gen_10000_8_s0")
    ids, adj, rp, col = fixture_csr(rec)
    a = oracle.c_color(rp, col, "A")
    assert list(a["round_U"]) == [9958, 9950, 9901, 9677, 8795, 6679, 3598, 1004, 113, 6, 0]
    assert a["max_color"] + 1 == 7
    sha = hashlib.sha256(_json.dumps([int(x) for x in a["colors"]]).encode()).hexdigest()[:16]
    assert sha == "246f30bd6a85cfa7"
    b = oracle.c_color(rp, col, "B")
    assert list(b["round_U"]) == [9958, 7243, 4256, 1670, 208, 1, 0]
    assert b["max_color"] + 1 == 6
    sha = hashlib.sha256(_json.dumps([int(x) for x in b["colors"]]).encode()).hexdigest()[:16]
    assert sha == "e36468939cca8079"
