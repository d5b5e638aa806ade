"""GPU parity: libgcolor.so (through the C-ABI) against the CPU oracle and the golden set.

Bit-exact for everything (integer work): final colours, per-round uncoloured /
proposer / accepted counts, max proposal per round, the round each vertex was coloured,
bounded-attempt failure round / count / snapshot, validation counts.
"""
import hashlib
import io
import json
import os
import random
import sys

import numpy as np
import pytest

from conftest import fixture_csr, golden_names, load_golden

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _dg():
    from gcolor_amd.engine import DeviceGraph
    return DeviceGraph


def assert_same_run(g, o, check_rounds=True):
    assert g.status == o["status"]
    assert np.array_equal(g.colors, o["colors"])
    if check_rounds:
        assert list(g.round_U) == list(o["round_U"])
        assert list(g.round_F) == list(o["round_F"])
        assert list(g.round_maxmex) == list(o["round_maxmex"])
        assert list(g.round_accepted) == list(o["round_accepted"])
        assert list(g.round_seeds) == list(o["round_seeds"])
        assert np.array_equal(g.colored_round, o["colored_round"])
    assert g.reseeds == o["reseeds"]
    if g.status == oracle.FAILED:
        assert (g.fail_round, g.fail_count) == (o["fail_round"], o["fail_count"])


GOLD_A = [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]]


@pytest.mark.parametrize("name", GOLD_A)
def test_golden_graphs_unbounded_and_bounded(name):
    rec = load_golden(name)
    ids, adj, rp, col = fixture_csr(rec)
    with _dg().from_csr(rp, col) as dg:
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert_same_run(g, o)
        run = rec["variants"]["A"]["run"]
        if run.get("colors") is not None:  # reference terminated: direct golden check too
            assert list(g.colors) == run["colors"]
            assert list(g.round_U) == run["rounds_U"]
        for k in range(0, int(o["max_color"]) + 2):
            assert_same_run(dg.color("A", num_colors=k), oracle.c_color(rp, col, "A", k=k))
        assert dg.validate(g.colors) == oracle.c_validate(rp, col, o["colors"])
        assert dg.validate() == oracle.c_validate(rp, col, o["colors"])  # device-resident result
        s = oracle.c_color(rp, col, "A", e1=False)
        gs = dg.color("A", e1=False)
        assert gs.status == s["status"] and np.array_equal(gs.colors, s["colors"])


CLI_CASES = [n for n in golden_names() if not load_golden(n)["variants"]["A"]["cli"]["hang"]
             and not load_golden(n)["variants"]["A"]["cli"].get("exception")]


@pytest.mark.parametrize("name", CLI_CASES)
def test_cli_end_to_end_matches_reference(name, tmp_path):
    from gcolor_amd import cli
    rec = load_golden(name)
    cli_rec = rec["variants"]["A"]["cli"]
    gpath = tmp_path / "g.json"
    with open(gpath, "w") as f:
        json.dump([{"id": i, "neighbors": nb, "color": -1} for i, nb in rec["graph"]], f, indent=4)
    argv = [a for a in cli_rec["argv"]]
    if "--input" in argv:
        argv[argv.index("--input") + 1] = str(gpath)
    else:  # generation mode: seed the global RNG like make_golden did
        argv += ["--seed", str(rec["params"]["seed"])]
        argv[argv.index("--output-graph") + 1] = str(tmp_path / "gen.json")
    out_c = tmp_path / "c.json"
    argv[argv.index("--output-coloring") + 1] = str(out_c)
    buf = io.StringIO()
    code = 0
    try:
        cli.main(argv + ["--compat-output"], out=buf)
    except SystemExit as e:
        code = e.code
    assert (code or 0) == cli_rec["exit"]
    lines = buf.getvalue().splitlines()
    norm = [("Iteration time: <t> seconds" if ln.startswith("Iteration time") else
             "Total execution time: <t> seconds" if ln.startswith("Total execution time") else ln) for ln in lines]
    assert norm == cli_rec["stdout"]
    if "output_sha256" in cli_rec:
        assert hashlib.sha256(out_c.read_bytes()).hexdigest() == cli_rec["output_sha256"]
        # default mode writes the valid colouring instead
        out_v = tmp_path / "v.json"
        argv[argv.index("--output-coloring") + 1] = str(out_v)
        cli.main(argv, out=io.StringIO())
        data = json.loads(out_v.read_text())
        assert [d["color"] for d in data] == rec["variants"]["A"]["run"]["colors"]


def _random_directed(n, m, seed, selfloops=True):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    if not selfloops:
        keep = src != dst
        src, dst = src[keep], dst[keep]
    order = np.argsort(src, kind="stable")
    src, dst = src[order], dst[order]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


@pytest.mark.parametrize("seed", range(6))
def test_directed_multigraphs_with_selfloops(seed):
    """Asymmetric lists, duplicates and self-loops keep the reference's directed semantics."""
    rp, col = _random_directed(3000, 9000, seed)
    with _dg().from_csr(rp, col) as dg:
        assert not dg.symmetric
        assert_same_run(dg.color("A"), oracle.c_color(rp, col, "A"))
        o = oracle.c_color(rp, col, "A")
        for k in (1, 2, int(o["max_color"])):
            assert_same_run(dg.color("A", num_colors=k), oracle.c_color(rp, col, "A", k=k))


@pytest.mark.parametrize("n,d,seed", [(200_000, 16, 1), (100_000, 8, 2), (50_000, 40, 3)])
def test_uniform_native_generator_graphs(n, d, seed):
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(n, d, seed)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("A")
        o = oracle.c_color(rp, col, "A")
        assert_same_run(g, o)
        assert dg.validate() == (0, 0)


@pytest.mark.parametrize("scale", [8, 10, 12, 14])
def test_rmat_graphs(scale):
    """Power-law: hubs (workgroup path), mex >= 64 (wide path), many small components (E1)."""
    DG = _dg()
    with DG.rmat(scale, 16, seed=scale) as dg:
        rp, col = dg.export()
        assert oracle_is_symmetric_simple(rp, col)
        g = dg.color("A")
        o = oracle.c_color(rp, col, "A")
        assert_same_run(g, o)
        assert dg.validate() == (0, 0)


def oracle_is_symmetric_simple(rp, col):
    n = len(rp) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    a = src * n + col
    b = col.astype(np.int64) * n + src
    return (not np.any(src == col)) and np.array_equal(np.sort(a), np.sort(b)) and np.unique(a).size == a.size


@pytest.mark.parametrize("dims", [(8, 8, 8), (16, 8, 4), (24, 24, 24)])
def test_mesh_graphs(dims):
    DG = _dg()
    with DG.mesh(*dims) as dg:
        rp, col = dg.export()
        g = dg.color("A")
        o = oracle.c_color(rp, col, "A")
        assert_same_run(g, o)
        assert g.max_color + 1 == 2   # wavefront 2-colours the bipartite mesh


def test_heavy_vertices_and_wide_mex():
    """A clique of 150 (mex up to 149) joined to a hub of degree 6000 (> GC_HEAVY_T)."""
    n = 150 + 6000
    adj = [[] for _ in range(n)]
    for i in range(150):
        for j in range(150):
            if i != j:
                adj[i].append(j)
    for leaf in range(150, n):
        adj[0].append(leaf)
        adj[leaf].append(0)
    for leaf in range(151, n, 7):  # some leaf-leaf edges
        adj[leaf].append(leaf - 1)
        adj[leaf - 1].append(leaf)
    from gcolor_amd.graphio import csr_from_adjacency
    rp, col = csr_from_adjacency(adj)
    with _dg().from_csr(rp, col) as dg:
        g = dg.color("A")
        o = oracle.c_color(rp, col, "A")
        assert_same_run(g, o)
        assert o["max_color"] >= 100


def test_empty_and_edgeless():
    DG = _dg()
    rp = np.zeros(4, np.int64)
    col = np.zeros(0, np.int32)
    with DG.from_csr(rp, col) as dg:
        g = dg.color("A")
        assert g.ok and list(g.colors) == [0, 0, 0] and list(g.round_U) == [0]


def test_reference_generator_10000_seeds():
    """random.seed(s); Graph(10000, 8) for s = 0..5 (golden) -- E1 seeds 1,2,3,5."""
    from gcolor_amd.generators import reference_csr
    for s in range(6):
        rp, col = reference_csr(10000, 8, random.Random(s))
        with _dg().from_csr(rp, col, symmetric=True) as dg:
            assert_same_run(dg.color("A"), oracle.c_color(rp, col, "A"))


def test_repeat_runs_are_identical():
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(300_000, 16, 9)
    with _dg().from_csr(rp, col, symmetric=True) as dg:
        a = dg.color("A")
        for _ in range(3):
            b = dg.color("A", kernel_timing=True)
            assert np.array_equal(a.colors, b.colors) and list(a.round_U) == list(b.round_U)
        assert b.kernels["propose"]["ms"] > 0


def _check_partition(dg):
    rp, col = dg.export()
    nl = dg.lower_counts()
    deg = np.diff(rp)
    n = len(rp) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    lower = (deg[col] < deg[src]) | ((deg[col] == deg[src]) & (col < src))
    pos = np.arange(len(col), dtype=np.int64) - rp[src]
    head = pos < nl[src]
    assert np.array_equal(lower, head), "rows must list exactly their lower-rank neighbours first"


def _expected_layout(rp, col):
    """The rank partition as gc_prep.hip states it, restated on the host: every row stably
    split into [lower degree | equal degree, earlier position | higher degree, earlier position
    | the rest] (coloring.py:64's (deg, pos) order: the first two classes are the lower ranks;
    the middle two are variant B's admission range, the last its eviction range)."""
    deg = np.diff(rp)
    n = len(rp) - 1
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    du, dv = deg[col], deg[src]
    early = col < src
    cls = np.where(du < dv, 0, np.where(early & (du == dv), 1, np.where(early, 2, 3)))
    order = np.argsort(src * 4 + cls, kind="stable")
    nlow = np.bincount(src, weights=(cls < 2), minlength=n).astype(np.int64)
    neq = np.bincount(src, weights=(cls == 1), minlength=n).astype(np.int64)
    return col[order], nlow, neq


def _heavy_graph(seed):
    """Rows past the tile geometry (2048 keys per tile, segments of 4096 entries): a few rows
    of 2049..20000 entries, runs of empty rows, duplicates and self-loops, directed."""
    rng = np.random.default_rng(seed)
    n = 30000
    deg = rng.integers(0, 12, n)
    deg[rng.integers(0, n, 3000)] = 0
    deg[[5, 6, 777, 20000, n - 1]] = [2049, 4096, 4097, 20000, 9000]
    deg[100:2100] = 0  # a long run of isolated rows inside a tile window
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(deg)
    col = rng.integers(0, n, rp[-1]).astype(np.int32)
    col[rp[5]:rp[5] + 100] = 5  # self-loops
    return rp, col


@pytest.mark.parametrize("kind", ["golden", "directed", "heavy", "heavy2"])
def test_partition_is_the_stable_three_class_split(kind):
    """Graph creation writes every row as the stable [lower deg | equal deg & earlier | rest]
    split of the input row -- tiles, segmented rows and empty rows alike (gc_prep.hip)."""
    DG = _dg()
    if kind == "golden":
        ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s0"))
    elif kind == "directed":
        rp, col = _random_directed(2000, 9000, 7)
    else:
        rp, col = _heavy_graph(1 if kind == "heavy" else 2)
    exp, nlow, neq = _expected_layout(rp, col)
    with DG.from_csr(rp, col) as dg:
        rp2, col2 = dg.export()
        assert np.array_equal(rp, rp2)
        assert np.array_equal(col2, exp)
        assert np.array_equal(dg.lower_counts(), nlow)
        # the same from a device-resident CSR (rows read in place)
        import torch
        d_rp = torch.from_numpy(rp).cuda()
        d_col = torch.from_numpy(col).cuda()
        torch.cuda.synchronize()
        with DG.from_device(d_rp.data_ptr(), d_col.data_ptr(), len(rp) - 1, len(col)) as dg2:
            assert np.array_equal(dg2.export()[1], exp)
            assert np.array_equal(dg2.lower_counts(), nlow)
            out_rp = torch.empty_like(d_rp)
            out_col = torch.empty_like(d_col)
            dg2.export_device(out_rp.data_ptr(), out_col.data_ptr())
            assert np.array_equal(out_col.cpu().numpy(), exp) and np.array_equal(out_rp.cpu().numpy(), rp)
        # the CSR still being written on a side stream, no host wait: the creation is ordered
        # after that stream by an event (gc_set_input_stream)
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            s_rp = torch.zeros_like(d_rp)
            s_col = torch.zeros_like(d_col)
            s_rp.copy_(d_rp)
            s_col.copy_(d_col)
        with DG.from_device(s_rp.data_ptr(), s_col.data_ptr(), len(rp) - 1, len(col), stream=side.cuda_stream) as dg3:
            assert np.array_equal(dg3.export()[1], exp)
        # validation over tiles and segmented rows, host and device colours
        rng = np.random.default_rng(3)
        for ncol in (1, 3, 50):
            cols = rng.integers(-1, ncol, len(rp) - 1).astype(np.int32)
            assert dg.validate(cols) == oracle.c_validate(rp, col, cols)


def test_create_device_rejects_bad_input():
    from gcolor_amd import _native as nat
    import torch
    DG = _dg()
    rp = np.array([0, 2, 3], np.int64)
    col = np.array([1, 5, 0], np.int32)  # 5 is out of range
    with pytest.raises(nat.GcolorError):
        DG.from_device(torch.from_numpy(rp).cuda().data_ptr(), torch.from_numpy(col).cuda().data_ptr(), 2, 3)
    rp_bad = torch.from_numpy(np.array([0, 3, 2], np.int64)).cuda()
    col_ok = torch.from_numpy(np.array([1, 0, 1], np.int32)).cuda()
    with pytest.raises(nat.GcolorError):
        DG.from_device(rp_bad.data_ptr(), col_ok.data_ptr(), 2, 3)


@pytest.mark.parametrize("kind", ["golden", "directed", "rmat", "mesh"])
def test_rows_list_lower_rank_neighbours_first(kind):
    """Graph creation stores each row lower-rank-first (rank = (deg, pos), coloring.py:64)
    without changing its multiset; nlow counts the head."""
    DG = _dg()
    if kind == "golden":
        ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s0"))
    elif kind == "directed":
        rp, col = _random_directed(2000, 9000, 7)
    if kind in ("golden", "directed"):
        with DG.from_csr(rp, col) as dg:
            rp2, col2 = dg.export()
            assert np.array_equal(rp, rp2)
            for v in range(len(rp) - 1):
                assert sorted(col[rp[v]:rp[v + 1]]) == sorted(col2[rp[v]:rp[v + 1]])
            _check_partition(dg)
    elif kind == "rmat":
        with DG.rmat(12, 16, seed=3) as dg:
            _check_partition(dg)
    else:
        with DG.mesh(9, 7, 5) as dg:
            _check_partition(dg)
