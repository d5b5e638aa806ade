"""GPU parity of variant B (coloring_optimized.py) through the C-ABI.

Bit-exact against the CPU oracle (oracle/gcolor_oracle.c, variant 1) and the golden
vectors recorded by running the reference's coloring_optimized.py: final colours,
per-round uncoloured / proposer / accepted counts, max proposal, the round each vertex
was coloured, bounded-attempt failure round / count / snapshot.  The arrival-order fold
(coloring_optimized.py:120-126, 168-200) runs as dependency-ordered admission / eviction
passes (csrc/gc_variant_b.hip); these cases drive long dependency chains (hubs, cliques,
directed lists with self-loops and duplicates) through it.
"""
import io
import json
import os
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from test_gpu_parity import _random_directed, assert_same_run  # noqa: E402

pytestmark = pytest.mark.gpu


def _dg():
    from gcolor_amd.engine import DeviceGraph
    return DeviceGraph


GOLD_B = [n for n in golden_names() if "B" in load_golden(n)["variants"]
          and "load_error" not in load_golden(n)["variants"]["B"]["run"]]


@pytest.mark.parametrize("name", GOLD_B)
def test_golden_graphs_variant_b(name):
    rec = load_golden(name)
    ids, adj, rp, col = fixture_csr(rec)
    with _dg().from_csr(rp, col) as dg:
        o = oracle.c_color(rp, col, "B")
        g = dg.color("B")
        assert_same_run(g, o)
        run = rec["variants"]["B"]["run"]
        if run.get("colors") is not None:  # the reference terminated: direct golden check too
            assert list(g.colors) == run["colors"]
            assert list(g.round_U) == run["rounds_U"]
            assert list(g.colored_round) == run["colored_round"]
        for k in range(0, int(o["max_color"]) + 2):
            assert_same_run(dg.color("B", num_colors=k), oracle.c_color(rp, col, "B", k=k))


def test_shipped_colors_json_is_the_failed_k2_snapshot():
    """The reference's colors.json == variant B's failed k=2 snapshot."""
    rec = load_golden("graph_json")
    ids, adj, rp, col = fixture_csr(rec)
    with _dg().from_csr(rp, col) as dg:
        g = dg.color("B", num_colors=2)
        assert not g.ok
        assert list(g.colors) == rec["variants"]["B"]["cli"]["output_colors"] == [0, 0, 1, -1, 1, -1, 0, 1, 1, 1]


def test_survey_pins_seed0_10000_variant_b():
    """Known-answer pin from SURVEY.md §8a (random.seed(0); Graph(10000, 8)), variant B."""
    rec = load_golden("gen_10000_8_s0")
    ids, adj, rp, col = fixture_csr(rec)
    with _dg().from_csr(rp, col) as dg:
        g = dg.color("B")
        assert list(g.round_U) == [9958, 7243, 4256, 1670, 208, 1, 0]
        assert g.max_color + 1 == 6


@pytest.mark.parametrize("seed", range(4))
def test_directed_multigraphs_with_selfloops_variant_b(seed):
    rp, col = _random_directed(3000, 9000, seed)
    with _dg().from_csr(rp, col) as dg:
        o = oracle.c_color(rp, col, "B")
        assert_same_run(dg.color("B"), o)
        for k in (0, 1, 2, int(o["max_color"])):
            assert_same_run(dg.color("B", num_colors=k), oracle.c_color(rp, col, "B", k=k))


@pytest.mark.parametrize("n,d,seed", [(200_000, 16, 1), (50_000, 40, 3)])
def test_uniform_graphs_variant_b(n, d, seed):
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(n, d, seed)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("B")
        assert_same_run(g, oracle.c_color(rp, col, "B"))
        assert dg.validate() == (0, 0)


@pytest.mark.parametrize("scale", [8, 12])
def test_rmat_graphs_variant_b(scale):
    with _dg().rmat(scale, 16, seed=scale) as dg:
        rp, col = dg.export()
        g = dg.color("B")
        assert_same_run(g, oracle.c_color(rp, col, "B"))
        assert dg.validate() == (0, 0)


def test_heavy_vertices_and_wide_mex_variant_b():
    n = 150 + 6000
    adj = [[] for _ in range(n)]
    for i in range(150):
        for j in range(150):
            if i != j:
                adj[i].append(j)
    for leaf in range(150, n):
        adj[0].append(leaf)
        adj[leaf].append(0)
    for leaf in range(151, n, 7):
        adj[leaf].append(leaf - 1)
        adj[leaf - 1].append(leaf)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    with _dg().from_csr(rp, col) as dg:
        o = oracle.c_color(rp, col, "B")
        assert_same_run(dg.color("B"), o)
        assert o["max_color"] >= 100


@pytest.mark.parametrize("hub_t,hub_w", [("0", "128"), ("64", "1"), ("512", "4"), ("off", "128")])
def test_variant_b_hub_bitmaps(monkeypatch, hub_t, hub_w):
    """Variant B proposes through the hubs' pushed forbidden-colour bitmaps: every threshold,
    a bitmap too small for the colours (row-scan fallback) and hubs off agree with the oracle."""
    monkeypatch.setenv("GC_HUB_T", hub_t)
    monkeypatch.setenv("GC_HUB_W", hub_w)
    with _dg().rmat(13, 16, seed=5) as dg:
        rp, col = dg.export()
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))
    n = 40 + 3000
    adj = [[] for _ in range(n)]
    for i in range(40):  # a clique of hubs (colours past a 1-word bitmap), each with leaves
        adj[i] += [j for j in range(40) if j != i]
    for leaf in range(40, n):
        hub = leaf % 40
        adj[hub].append(leaf)
        adj[leaf].append(hub)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    with _dg().from_csr(rp, col) as dg:
        o = oracle.c_color(rp, col, "B")
        assert_same_run(dg.color("B"), o)
        assert_same_run(dg.color("B", num_colors=int(o["max_color"])), oracle.c_color(rp, col, "B", k=int(o["max_color"])))


FOLD_SETTINGS = [
    {"GC_B_ASYNC": "0"},                                                  # full-grid passes only
    {},                                                                   # k_b_async where there are hubs
    {"GC_B_ASYNC": "1"},                                                  # k_b_async on every graph
    {"GC_B_ASYNC": "1", "GC_B_ASYNC_K": "1"},                             # one full pass first
    {"GC_B_ASYNC": "1", "GC_B_ASYNC_K": "3"},
    {"GC_B_ASYNC": "1", "GC_ASYNC_BUDGET_US": "0"},                       # gives up at once: hands back to passes
    {"GC_B_ASYNC": "1", "GC_B_ASYNC_BPC": "1"},                           # one workgroup per CU
    {"GC_B_PIPE": "0"},                                                   # one host wait per round, no pipelining
    {"GC_B_PIPE": "0", "GC_B_ASYNC": "0"},
    {"GC_B_PIPE": "0", "GC_B_ASYNC": "1", "GC_ASYNC_BUDGET_US": "0"},
    {"GC_B_ASYNC": "1", "GC_B_WATCH": "0"},                               # admission cursors off: full rescans
    {"GC_B_ASYNC": "1", "GC_B_WATCH": "64", "GC_B_AWIN": "1"},            # one entry per window, rare rescans
    {"GC_B_ASYNC": "1", "GC_B_ASYNC_K": "1", "GC_B_WATCH": "2", "GC_B_AWIN": "3"},
    {"GC_B_ASYNC": "1", "GC_B_RESIDENT": "0"},                            # the fold's non-resident form only
    {"GC_B_ASYNC": "1", "GC_B_REFSKIP": "0"},                             # refused admissions read on
    {"GC_B_ASYNC": "1", "GC_B_RESIDENT": "0", "GC_B_REFSKIP": "0"},
    {"GC_B_ASYNC": "1", "GC_B_RESIDENT": "1", "GC_ASYNC_BUDGET_US": "0"},  # resident form's stop-and-write-back
]


@pytest.mark.parametrize("env", FOLD_SETTINGS, ids=["grid", "default", "async", "async_k1", "async_k3", "async_abort",
                                                    "async_bpc1", "nopipe", "nopipe_grid", "nopipe_abort",
                                                    "cursor_off", "cursor_w1", "cursor_k1_w3", "resident_off",
                                                    "refskip_off", "resident_refskip_off", "resident_abort"])
def test_variant_b_fold(monkeypatch, env):
    """The fold's passes on the full grid, the asynchronous fold where there are hubs (the
    default), on every graph after 0, 1 or 3 full passes, and forced to hand back at once --
    pipelined rounds (the default: the commit decides done / failed / unfinished) and one
    host wait per round (GC_B_PIPE=0) -- every run equal to the oracle."""
    for k in ("GC_B_ASYNC", "GC_B_ASYNC_K", "GC_ASYNC_BUDGET_US", "GC_B_ASYNC_BPC", "GC_B_PIPE", "GC_B_WATCH", "GC_B_AWIN",
              "GC_B_RESIDENT", "GC_B_REFSKIP"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with _dg().rmat(13, 16, seed=5) as dg:
        rp, col = dg.export()
        o = oracle.c_color(rp, col, "B")
        assert_same_run(dg.color("B"), o)
        assert_same_run(dg.color("B", num_colors=int(o["max_color"]) // 2), oracle.c_color(rp, col, "B", k=int(o["max_color"]) // 2))
    rp, col = _random_directed(3000, 9000, 7)
    with _dg().from_csr(rp, col) as dg:
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))
    n = 150 + 6000  # a 150-clique whose first vertex is a hub of 6000 leaves (heavy admissions, wide mex)
    adj = [[] for _ in range(n)]
    for i in range(150):
        adj[i] += [j for j in range(150) if j != i]
    for leaf in range(150, n):
        adj[0].append(leaf)
        adj[leaf].append(0)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    with _dg().from_csr(rp, col) as dg:
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(50_000, 40, 3)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))
    h = 2050  # K_{h,h}: every row is h equal-degree entries, past GC_B_HEAVY: heavy admissions only
    rp = np.arange(2 * h + 1, dtype=np.int64) * h
    col = np.concatenate([np.tile(np.arange(h, 2 * h, dtype=np.int32), h), np.tile(np.arange(h, dtype=np.int32), h)])
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))


def test_mesh_and_edgeless_variant_b():
    DG = _dg()
    with DG.mesh(16, 8, 4) as dg:
        rp, col = dg.export()
        assert_same_run(dg.color("B"), oracle.c_color(rp, col, "B"))
    rp = np.zeros(4, np.int64)
    col = np.zeros(0, np.int32)
    with DG.from_csr(rp, col) as dg:
        g = dg.color("B")
        assert g.ok and list(g.colors) == [0, 0, 0] and list(g.round_U) == [0]


CLI_B = [n for n in GOLD_B if not load_golden(n)["variants"]["B"]["cli"]["hang"]
         and not load_golden(n)["variants"]["B"]["cli"].get("exception")]


@pytest.mark.parametrize("name", CLI_B[::4])
def test_cli_variant_b_matches_reference(name, tmp_path):
    """`--variant B` reproduces coloring_optimized.py's transcript and output file."""
    import hashlib
    from gcolor_amd import cli
    rec = load_golden(name)
    cli_rec = rec["variants"]["B"]["cli"]
    gpath = tmp_path / "g.json"
    with open(gpath, "w") as f:
        json.dump([{"id": i, "neighbors": nb, "color": -1} for i, nb in rec["graph"]], f, indent=4)
    argv = list(cli_rec["argv"])
    if "--input" in argv:
        argv[argv.index("--input") + 1] = str(gpath)
    else:
        argv += ["--seed", str(rec["params"]["seed"])]
        argv[argv.index("--output-graph") + 1] = str(tmp_path / "gen.json")
    out_c = tmp_path / "c.json"
    argv[argv.index("--output-coloring") + 1] = str(out_c)
    buf = io.StringIO()
    code = 0
    try:
        cli.main(argv + ["--variant", "B", "--compat-output"], out=buf)
    except SystemExit as e:
        code = e.code
    assert (code or 0) == cli_rec["exit"]
    lines = buf.getvalue().splitlines()
    norm = [("Iteration time: <t> seconds" if ln.startswith("Iteration time") else
             "Total execution time: <t> seconds" if ln.startswith("Total execution time") else ln) for ln in lines]
    assert norm == cli_rec["stdout"]
    if "output_sha256" in cli_rec:
        assert hashlib.sha256(out_c.read_bytes()).hexdigest() == cli_rec["output_sha256"]


@pytest.mark.parametrize("env", [{}, {"GC_B_ASYNC": "0"}], ids=["async", "passes"])
def test_rmat20_variant_b_against_oracle(monkeypatch, env):
    """R-MAT-20 (10^6 vertices, hubs of 10^4 entries, ~200 rounds): variant B's fold at a size
    where the asynchronous fold spreads every round over thousands of waves, and the full-grid
    passes -- every colour and per-round record equal to the C oracle's (variant 1)."""
    for k in ("GC_B_ASYNC", "GC_B_ASYNC_K", "GC_B_ASYNC_BPC", "GC_B_RESIDENT", "GC_B_REFSKIP"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with _dg().rmat(20, 16, seed=1) as dg:
        rp, col = dg.export()
        g = dg.color("B")
        assert_same_run(g, oracle.c_color(rp, col, "B"))
        assert dg.validate() == (0, 0)


@pytest.mark.parametrize("bpc", ["7", "8"])
def test_fold_past_six_per_cu_requested(monkeypatch, bpc):
    """variant B's asynchronous fold asked for 7 / 8 workgroups per CU on R-MAT-20
    (round 5's cliff: 10-13 give-ups a colouring) -- no give-up, the oracle's colouring.  The
    default build is compiled for 6 waves per SIMD (80 VGPRs), so the grid is capped at the
    residency the probe measures (6); builds for 7 and 8 (-DGC_B_WPE=7/8, resident caps 640 /
    512) ran every workgroup resident with no give-up either (profiles/r06/f, g)."""
    for k in ("GC_B_ASYNC", "GC_B_ASYNC_K", "GC_ASYNC_BUDGET_US", "GC_B_RESIDENT", "GC_B_REFSKIP"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GC_B_ASYNC_BPC", bpc)
    with _dg().rmat(20, 16, seed=5) as dg:
        rp, col = dg.export()
        g = dg.color("B")
        assert g.async_aborts == 0
        assert_same_run(g, oracle.c_color(rp, col, "B"))


def test_async_grids_sized_from_measured_residency(monkeypatch):
    """The asynchronous kernels' grids (variant B's fold k_b_async, variant A's k_sweep_async)
    are capped at the workgroups measured resident (gc_residency_probe); any requested grid,
    including 8 per CU -- round 4's cliff -- gives the same colouring.  (Round 5 measured every
    workgroup resident at 8 per CU, so the cliff is not residency: from 7 per CU variant B's fold
    gives up 10-13 times per R-MAT-20 colouring, profiles/r05/e; the default stays 4.)"""
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(20, 16, seed=5) as dg:
        ref_b = dg.color("B")
        ref_a = dg.color("A")
        assert ref_b.async_aborts == 0 and ref_a.async_aborts == 0
        for bpc in ("6", "8"):
            monkeypatch.setenv("GC_B_ASYNC_BPC", bpc)
            monkeypatch.setenv("GC_ASYNC_BPC", bpc)
            b = dg.color("B")
            a = dg.color("A")
            assert np.array_equal(b.colors, ref_b.colors) and list(b.round_U) == list(ref_b.round_U)
            assert np.array_equal(a.colors, ref_a.colors) and list(a.round_U) == list(ref_a.round_U)
