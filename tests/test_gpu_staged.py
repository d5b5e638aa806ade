"""Staged GPU tests (marker gpu_staged, NOT selected by -m gpu): opt-in paths written in a
round whose GPU access had closed, to be run with `pytest -m gpu_staged` on the next box and
promoted to `gpu` once green (tools/gpu_plan_r04.sh runs them in order).
Run: GC_RUN_STAGED=1 python -m pytest tests/test_gpu_staged.py -m gpu_staged -x -v [-k GROUP]

* b_async: variant B's asynchronous fold (GC_B_ASYNC=1, k_b_async) on every variant-B parity
  case of tests/test_gpu_variant_b.py, with the normal budget and a zero one.
* async_jp_without_hubs: the asynchronous JP on hub-less graphs (GC_ASYNC=2), the path that
  faulted at 10M vertices in round 3, small first, then C2.
* async_resolve: the round's first JP sweep inside k_sweep_async (GC_ASYNC_RESOLVE=1).
* big_close: k_commit_big closes the round (GC_BIG_CLOSE=1).
* test_graphs_: each round's launches replayed as a hipGraph (GC_GRAPHS=1).
* small_grid: small rounds' resolve / commit grids capped (GC_GRID_SMALL).
(overflow_tree / under_ticket_close, resume and hybrid moved to tests/test_gpu_resume.py in
round 4, after their first green run.)
* validate_c8: the validation from the byte mirror (GC_VALIDATE_C8=1).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import test_gpu_variant_b as vb  # noqa: E402
from oracle import oracle  # noqa: E402

# selected only by `-m gpu_staged` with GC_RUN_STAGED=1 (the CPU suite's -m "not gpu" skips them)
pytestmark = [pytest.mark.gpu_staged,
              pytest.mark.skipif(not os.environ.get("GC_RUN_STAGED"), reason="staged: GC_RUN_STAGED=1 -m gpu_staged")]

B_ENVS = [{"GC_B_ASYNC": "1"}, {"GC_B_ASYNC": "1", "GC_ASYNC_BUDGET_US": "0"}]
B_IDS = ["basync", "basync_abort"]


@pytest.fixture(params=B_ENVS, ids=B_IDS)
def benv(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


@pytest.mark.parametrize("name", vb.GOLD_B[::2])
def test_b_async_golden(benv, name):
    vb.test_golden_graphs_variant_b(name)


def test_b_async_pins(benv):
    vb.test_shipped_colors_json_is_the_failed_k2_snapshot()
    vb.test_survey_pins_seed0_10000_variant_b()


@pytest.mark.parametrize("seed", range(4))
def test_b_async_directed(benv, seed):
    vb.test_directed_multigraphs_with_selfloops_variant_b(seed)


@pytest.mark.parametrize("n,d,seed", [(200_000, 16, 1), (50_000, 40, 3)])
def test_b_async_uniform(benv, n, d, seed):
    vb.test_uniform_graphs_variant_b(n, d, seed)


@pytest.mark.parametrize("scale", [8, 12])
def test_b_async_rmat(benv, scale):
    vb.test_rmat_graphs_variant_b(scale)


def test_b_async_heavy(benv):
    vb.test_heavy_vertices_and_wide_mex_variant_b()


def test_b_async_rmat24_matches_passes(monkeypatch):
    """C3 under variant B: the asynchronous fold equals the host passes, round for round."""
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(24, 16, seed=1) as dg:
        ref = dg.color("B")
        monkeypatch.setenv("GC_B_ASYNC", "1")
        g = dg.color("B")
        assert g.async_aborts == 0
        assert np.array_equal(g.colors, ref.colors)
        assert list(g.round_U) == list(ref.round_U) and list(g.round_accepted) == list(ref.round_accepted)


@pytest.mark.parametrize("n", [100_000, 1_000_000, 10_000_000])
def test_async_jp_without_hubs_uniform(monkeypatch, n):
    """GC_ASYNC=2 forces k_sweep_async on graphs with no hub (round 3: C2 at 10M faulted in
    the k_commit after it); against the synchronous sweeps."""
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    rp, col = uniform_csr(n, 16, 42)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        monkeypatch.setenv("GC_ASYNC", "0")
        ref = dg.color("A")
        monkeypatch.setenv("GC_ASYNC", "2")
        g = dg.color("A")
        assert np.array_equal(g.colors, ref.colors)
        assert list(g.round_U) == list(ref.round_U)


# --- the asynchronous first sweep (GC_ASYNC_RESOLVE=1: no k_resolve launch) ---------------
import test_gpu_hubs as hubs  # noqa: E402

R_ENVS = [{"GC_ASYNC_RESOLVE": "1"}, {"GC_ASYNC_RESOLVE": "1", "GC_ASYNC_BUDGET_US": "0"},
          {"GC_ASYNC_RESOLVE": "1", "GC_HUB_T": "2"}, {"GC_ASYNC_RESOLVE": "1", "GC_HUB_T": "0", "GC_ASYNC_BUDGET_US": "0"}]
R_IDS = ["ares", "ares_abort", "ares_T2", "ares_T0_abort"]


@pytest.fixture(params=R_ENVS, ids=R_IDS)
def renv(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


def test_async_resolve_generator_graphs(renv):
    hubs.test_reference_generator_graphs(renv)


@pytest.mark.parametrize("seed", range(3))
def test_async_resolve_directed(renv, seed):
    hubs.test_directed_multigraphs(renv, seed)


@pytest.mark.parametrize("scale", [9, 12])
def test_async_resolve_rmat(renv, scale):
    hubs.test_rmat(renv, scale)


def test_async_resolve_clique_star(renv):
    hubs.test_clique_and_star(renv)


def test_async_resolve_rmat24_matches(monkeypatch):
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(24, 16, seed=1) as dg:
        ref = dg.color("A")
        monkeypatch.setenv("GC_ASYNC_RESOLVE", "1")
        g = dg.color("A")
        assert g.async_aborts == 0
        assert np.array_equal(g.colors, ref.colors)
        for k in ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds"):
            assert list(getattr(g, k)) == list(getattr(ref, k)), k
        assert g.kernels["resolve"]["bytes"] == ref.kernels["resolve"]["bytes"]  # the first sweep's §8d credit


# --- the round closed by k_commit_big (GC_BIG_CLOSE=1: no k_close launch on graphs with big rows) ---
BC_ENVS = [{"GC_BIG_CLOSE": "1"}, {"GC_BIG_CLOSE": "1", "GC_BIGROW": "8"}, {"GC_BIG_CLOSE": "1", "GC_HUB_T": "0"},
           {"GC_BIG_CLOSE": "1", "GC_BIGROW": "8", "GC_BATCH_MAX": "1"}]
BC_IDS = ["bclose", "bclose_row8", "bclose_nohub", "bclose_row8_batch1"]


@pytest.fixture(params=BC_ENVS, ids=BC_IDS)
def bcenv(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


def test_big_close_generator_graphs(bcenv):
    hubs.test_reference_generator_graphs(bcenv)


@pytest.mark.parametrize("seed", range(3))
def test_big_close_directed(bcenv, seed):
    hubs.test_directed_multigraphs(bcenv, seed)


@pytest.mark.parametrize("scale", [9, 12])
def test_big_close_rmat(bcenv, scale):
    hubs.test_rmat(bcenv, scale)


@pytest.mark.parametrize("bigrow", ["0", "8", "64"])
@pytest.mark.parametrize("hub_t", ["0", "4", "1024"])
def test_big_close_commit_big_tiles(monkeypatch, bigrow, hub_t):
    monkeypatch.setenv("GC_BIG_CLOSE", "1")
    hubs.test_commit_big_tiles(monkeypatch, bigrow, hub_t)


def test_big_close_rmat24_matches(monkeypatch):
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(24, 16, seed=1) as dg:
        ref = dg.color("A")
        monkeypatch.setenv("GC_BIG_CLOSE", "1")
        g = dg.color("A")
        assert np.array_equal(g.colors, ref.colors)
        for k in ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds"):
            assert list(getattr(g, k)) == list(getattr(ref, k)), k
        assert dg.validate() == (0, 0)


# --- each round's launches captured once per shape in a hipGraph and replayed (GC_GRAPHS=1) ---
G_ENVS = [{"GC_GRAPHS": "1"}, {"GC_GRAPHS": "1", "GC_BATCH_MAX": "1"}, {"GC_GRAPHS": "1", "GC_ASYNC": "0"},
          {"GC_GRAPHS": "1", "GC_HUB_T": "off"}, {"GC_GRAPHS": "1", "GC_ASYNC_BUDGET_US": "0"}]
G_IDS = ["graphs", "graphs_batch1", "graphs_sync_jp", "graphs_nohub", "graphs_abort"]


@pytest.fixture(params=G_ENVS, ids=G_IDS)
def genv(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


def test_graphs_generator_graphs(genv):
    hubs.test_reference_generator_graphs(genv)


@pytest.mark.parametrize("seed", range(3))
def test_graphs_directed(genv, seed):
    hubs.test_directed_multigraphs(genv, seed)


@pytest.mark.parametrize("scale", [9, 12])
def test_graphs_rmat(genv, scale):
    hubs.test_rmat(genv, scale)


def test_graphs_uniform_and_mesh(genv):
    """Hub-less graphs: fused and closing commits, the big-round rebuild, E1 on the generator."""
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    rp, col = uniform_csr(300_000, 16, 7)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert np.array_equal(g.colors, o["colors"]) and list(g.round_U) == list(o["round_U"])
    with DeviceGraph.mesh(40, 32, 24) as dg:
        rp, col = dg.export()
        o = oracle.c_color(rp, col, "A")
        g = dg.color("A")
        assert np.array_equal(g.colors, o["colors"]) and list(g.round_U) == list(o["round_U"])


def test_graphs_rmat24_matches(monkeypatch):
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(24, 16, seed=1) as dg:
        ref = dg.color("A")
        monkeypatch.setenv("GC_GRAPHS", "1")
        g = dg.color("A")
        assert np.array_equal(g.colors, ref.colors)
        for k in ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds"):
            assert list(getattr(g, k)) == list(getattr(ref, k)), k
        print(f"R-MAT-24 device ms: direct {ref.device_ms:.1f}, graphs {g.device_ms:.1f}")


# --- small rounds on capped grids (GC_GRID_SMALL: resolve / commit / commit_big) ------------
S_ENVS = [{"GC_GRID_SMALL": "64"}, {"GC_GRID_SMALL": "1"}, {"GC_GRID_SMALL": "8", "GC_BIG_CLOSE": "1"},
          {"GC_GRID_SMALL": "8", "GC_HUB_T": "off", "GC_FUSE": "0"}]
S_IDS = ["small64", "small1", "small8_bclose", "small8_nohub_unfused"]


@pytest.fixture(params=S_ENVS, ids=S_IDS)
def senv(request, monkeypatch):
    for k, v in request.param.items():
        monkeypatch.setenv(k, v)
    return request.param


def test_small_grid_generator_graphs(senv):
    hubs.test_reference_generator_graphs(senv)


@pytest.mark.parametrize("seed", range(3))
def test_small_grid_directed(senv, seed):
    hubs.test_directed_multigraphs(senv, seed)


@pytest.mark.parametrize("scale", [9, 12])
def test_small_grid_rmat(senv, scale):
    hubs.test_rmat(senv, scale)


def test_small_grid_uniform_and_mesh(senv):
    test_graphs_uniform_and_mesh(senv)


def test_small_grid_rmat24_matches(monkeypatch):
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(24, 16, seed=1) as dg:
        ref = dg.color("A")
        for grid in ("128", "256"):
            monkeypatch.setenv("GC_GRID_SMALL", grid)
            g = dg.color("A")
            assert np.array_equal(g.colors, ref.colors)
            for k in ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds"):
                assert list(getattr(g, k)) == list(getattr(ref, k)), k
            print(f"R-MAT-24 device ms: default grids {ref.device_ms:.1f}, GC_GRID_SMALL={grid} {g.device_ms:.1f}")


# --- validation from the byte mirror (GC_VALIDATE_C8=1, the resident colouring) -------------
def test_validate_c8_matches(monkeypatch):
    """The resident colouring validated from c8 counts what the int colours count: after a full
    run, after a failed bounded run (uncoloured vertices), and after a resume from a state with
    planted conflicts (colours < 254 and >= 254, the byte mirror's BIG case)."""
    import torch
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(12, 16, seed=9) as dg:
        rp, col = dg.export()
        for k in (None, 3):
            g = dg.color("A", num_colors=k)
            monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
            ref = dg.validate()
            monkeypatch.setenv("GC_VALIDATE_C8", "1")
            assert dg.validate() == ref == tuple(oracle.c_validate(rp, col, g.colors))
        v = int(np.argmax(np.diff(rp)))  # the largest row: it has neighbours
        u = int(col[rp[v]])
        c = np.full(dg.n, -1, np.int32)
        c[v], c[u] = 300, 300  # a conflict past the byte mirror
        w = next(int(x) for x in col[rp[u]:rp[u + 1]] if int(x) not in (u, v))
        x = next((int(y) for y in col[rp[w]:rp[w + 1]] if int(y) not in (u, v, w)), None)
        c[w] = 5
        if x is not None:
            c[x] = 5  # a conflict below 254
        front = np.array(sorted(y for y in set(int(y) for y in col[rp[v]:rp[v + 1]]) if c[y] < 0), np.int32)
        ct, ft = torch.from_numpy(c).cuda(), torch.from_numpy(front if len(front) else np.zeros(1, np.int32)).cuda()
        torch.cuda.synchronize()
        g = dg.resume(ct.data_ptr(), ft.data_ptr(), len(front), 0)
        monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
        ref = dg.validate()
        monkeypatch.setenv("GC_VALIDATE_C8", "1")
        assert dg.validate() == ref == tuple(oracle.c_validate(rp, col, g.colors))
        assert ref[1] > 0

