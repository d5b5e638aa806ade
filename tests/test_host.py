"""Host-side logic of the drop-in (no GPU): generator, JSON I/O, transcript derivation.

The transcript derivation (gcolor_amd.cli.transcript) is fed with oracle runs here; on
the GPU the same function is fed with libgcolor.so runs (tests/test_gpu_parity.py).
"""
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

from gcolor_amd import cli, graphio  # noqa: E402
from gcolor_amd.generators import reference_graph  # noqa: E402

GEN = [n for n in golden_names() if n.startswith("gen_")]


@pytest.mark.parametrize("name", GEN)
def test_reference_generator_bit_identical(name):
    rec = load_golden(name)
    p = rec["params"]
    rng = random.Random(p["seed"])
    adj = reference_graph(p["node_count"], p["max_degree"], rng)
    assert [[i, a] for i, a in enumerate(adj)] == rec["graph"]


def test_cli_generation_graph_file_bytes(tmp_path):
    """--node-count/--max-degree/--output-graph path (coloring.py:182-187, graph.py:10-12)."""
    rec = load_golden("cli_generate_200_5_s7")
    random.seed(7)
    rp, col = graphio.csr_from_adjacency(reference_graph(200, 5))
    out = tmp_path / "g.json"
    graphio.write_graph_json(str(out), list(range(200)), rp, col)
    cli_rec = rec["variants"]["A"]["cli"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == cli_rec["graph_out_sha256"]


@pytest.mark.parametrize("name", [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]])
def test_json_roundtrip_and_output_bytes(name, tmp_path):
    rec = load_golden(name)
    gpath = tmp_path / "g.json"
    with open(gpath, "w") as f:
        json.dump([{"id": i, "neighbors": nb, "color": -1} for i, nb in rec["graph"]], f, indent=4)
    ids, rp, col = graphio.load_graph_json(str(gpath))
    ids2, _, rp2, col2 = fixture_csr(rec)
    assert list(ids) == list(ids2) and np.array_equal(rp, rp2) and np.array_equal(col, col2)
    for v, vr in rec["variants"].items():
        cli_rec = vr["cli"]
        if "output_sha256" not in cli_rec:
            continue
        out = tmp_path / f"c{v}.json"
        graphio.write_coloring_json(str(out), cli_rec["output_ids"], cli_rec["output_colors"])
        assert hashlib.sha256(out.read_bytes()).hexdigest() == cli_rec["output_sha256"]


def test_missing_neighbor_raises_keyerror(tmp_path):
    rec = load_golden("missing_neighbor")
    p = tmp_path / "g.json"
    p.write_text(json.dumps([{"id": i, "neighbors": nb, "color": -1} for i, nb in rec["graph"]]))
    with pytest.raises(KeyError) as ei:
        graphio.load_graph_json(str(p))
    assert f"Error loading graph: {ei.value}" == rec["variants"]["A"]["cli"]["stdout"][0]


class _R:
    def __init__(self, d):
        self.round_U = d["round_U"]
        self.round_maxmex = d["round_maxmex"]
        self.max_color = d["max_color"]
        self.fail_count = d["fail_count"]
        self.colors = d["colors"]


CLI_CASES = [(n, v) for n in golden_names() for v in load_golden(n)["variants"]
             if not load_golden(n)["variants"][v]["cli"]["hang"]
             and not load_golden(n)["variants"][v]["cli"].get("exception")
             and load_golden(n)["variants"][v]["cli"]["exit"] == 0]


@pytest.mark.parametrize("name,variant", CLI_CASES)
def test_transcript_from_single_run_matches_reference(name, variant):
    """One unbounded run + the failing attempt reproduce the reference's k-loop stdout."""
    rec = load_golden(name)
    cli_rec = rec["variants"][variant]["cli"]
    ids, adj, rp, col = fixture_csr(rec)
    argv = cli_rec["argv"]
    maxdeg_arg = int(argv[argv.index("--max-degree") + 1]) if "--max-degree" in argv else None
    K0 = maxdeg_arg + 1 if maxdeg_arg else max(len(a) for a in adj) + 1
    full = oracle.c_color(rp, col, variant)
    _, fail_k, _ = cli.attempt_plan(K0, full["round_maxmex"], full["max_color"])
    b = oracle.c_color(rp, col, variant, k=fail_k) if fail_k is not None else None
    lines, _, minimal = cli.transcript(K0, _R(full), 0.0, oracle.c_validate(rp, col, full["colors"]),
                                       _R(b) if b else None, 0.0,
                                       oracle.c_validate(rp, col, b["colors"]) if b else None)
    lines = [ln if not ln.startswith("Iteration time") else "Iteration time: <t> seconds" for ln in lines]
    lines += ["Total execution time: <t> seconds", f"Minimal number of colors: {minimal}"]
    assert lines == cli_rec["stdout"]
    assert list(b["colors"]) == cli_rec["output_colors"]


def test_attempt_plan_edge_cases():
    # nothing ever proposed (edgeless / self-loop seeds only): reference never ends
    assert cli.attempt_plan(1, [-1], 0) == ([1], None, 1)
    # K0 below the colours needed: first attempt fails (coloring.py:226-228)
    assert cli.attempt_plan(3, [1, 2, 3, 4], 4) == ([], 3, 4)
    assert cli.attempt_plan(6, [1, 2, 1, -1], 2) == ([6, 5, 4, 3], 2, 3)
