"""Multi-rank driver of the sharded engine (gcolor_amd.shard) on CPU.

The HIP phases are replaced by tests/shard_numpy.NumpyShard (same interface and delta
format); the driver, the exchange protocol and both transports are the product code.
Results must equal the single-partition oracle bit for bit: LFMIS under the global rank
(deg, pos) does not depend on the partition.
"""
import json
import os
import sys
import threading

import numpy as np
import pytest
import torch

from conftest import PKG_DIR, REPO, fixture_csr, free_port, golden_names, load_golden

sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402
from shard_numpy import DeferredNumpyShard, InflatedShard, NumpyShard, numpy_resume  # noqa: E402

from gcolor_amd import shard as sh  # noqa: E402


def _random_directed(n, m, seed):
    rng = np.random.default_rng(seed)
    src = np.sort(rng.integers(0, n, m))
    dst = rng.integers(0, n, m)
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


def run_threads(rp, col, parts, k=None, e1=True, deferred_ops=False, shard_cls=None, switch_below=None, calls=None,
                **kw):
    ranges = sh.balanced_ranges(rp, parts)
    hub = sh.ThreadHub(parts)
    out, err = [None] * parts, []

    def go(i):
        try:
            cls = shard_cls or (DeferredNumpyShard if deferred_ops else NumpyShard)
            ops = cls(rp, col, *ranges[i])
            comm = sh.ThreadTransport(hub, i)
            if switch_below is None:
                out[i] = sh.shard_color(ops, comm, k, e1, track_rounds=True, **kw)
            else:
                out[i] = sh.hybrid_color(ops, comm, numpy_resume(rp, col, calls if i == 0 else None), switch_below, k,
                                         e1, track_rounds=True, **kw)
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            hub.barrier.abort()

    ts = [threading.Thread(target=go, args=(i,)) for i in range(parts)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return out


def assert_matches_oracle(res, o):
    assert res.status == o["status"]
    assert np.array_equal(res.colors, o["colors"])
    assert np.array_equal(res.colored_round, o["colored_round"])
    for key in ("U", "F", "maxmex", "accepted", "seeds"):
        assert list(getattr(res, "round_" + key)) == list(o["round_" + key]), key
    assert res.reseeds == o["reseeds"]
    if res.status == oracle.FAILED:
        assert (res.fail_round, res.fail_count) == (o["fail_round"], o["fail_count"])


def test_balanced_ranges_cover_and_balance():
    rp = np.cumsum(np.r_[0, np.random.default_rng(0).integers(0, 50, 1000)])
    for parts in (1, 2, 3, 8):
        rs = sh.balanced_ranges(rp, parts)
        assert rs[0][0] == 0 and rs[-1][1] == 1000
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        w = [int(rp[hi] - rp[lo] + hi - lo) for lo, hi in rs]
        assert max(w) - min(w) <= 2 * (50 + 1)  # each boundary is off by at most one vertex
    assert sh.balanced_ranges(np.zeros(1, np.int64), 4) == [(0, 0)] * 4


GOLD = [n for n in golden_names() if "load_error" not in load_golden(n)["variants"]["A"]["run"]
        and len(load_golden(n)["graph"]) <= 1000]


@pytest.mark.parametrize("name", GOLD)
@pytest.mark.parametrize("parts", [2, 3])
def test_threads_match_oracle_on_golden_graphs(name, parts):
    ids, adj, rp, col = fixture_csr(load_golden(name))
    res = run_threads(rp, col, parts)
    o = oracle.c_color(rp, col, "A")
    for r in res:  # every rank holds the same result
        assert_matches_oracle(r, o)
    run = load_golden(name)["variants"]["A"]["run"]
    if run.get("colors") is not None:
        assert list(res[0].colors) == run["colors"]


@pytest.mark.parametrize("seed", range(4))
def test_threads_directed_selfloops_bounded_and_stalled(seed):
    rp, col = _random_directed(300, 900, seed)
    o = oracle.c_color(rp, col, "A")
    assert_matches_oracle(run_threads(rp, col, 3)[0], o)
    for k in (1, int(o["max_color"])):
        assert_matches_oracle(run_threads(rp, col, 2, k=k)[1], oracle.c_color(rp, col, "A", k=k))
    s = oracle.c_color(rp, col, "A", e1=False)
    r = run_threads(rp, col, 2, e1=False)[0]
    assert r.status == s["status"] and np.array_equal(r.colors, s["colors"])


@pytest.mark.parametrize("deferred_ops", [False, True])
@pytest.mark.parametrize("dense", [True, False, None])
@pytest.mark.parametrize("local_sweeps", [1, 3])
@pytest.mark.parametrize("inline", [4096, 5, 0])
def test_dense_seams_and_local_sweeps(dense, local_sweeps, inline, deferred_ops):
    """Slices of the proposal bytes instead of deltas, several JP sweeps between
    exchanges, and deltas that overflow the inline part of a seam's all-gather (a second
    exchange: the rest of the deltas, or slices) leave the result unchanged; so do the
    enqueue-only round end and the fused propose seam (deferred_ops), its misses included."""
    for seed in range(3):
        rp, col = _random_directed(400, 2000, 10 + seed)
        o = oracle.c_color(rp, col, "A")
        res = run_threads(rp, col, 3, dense=dense, local_sweeps=local_sweeps, inline=inline, inline_max=inline,
                          deferred_ops=deferred_ops)
        assert_matches_oracle(res[seed % 3], o)
        if dense:
            assert res[0].dense_exchanges > 0
        elif dense is False:
            assert res[0].dense_exchanges == 0
    ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s1"))
    assert_matches_oracle(run_threads(rp, col, 2, dense=dense, local_sweeps=local_sweeps, inline=inline, inline_max=inline,
                                      deferred_ops=deferred_ops)[1], oracle.c_color(rp, col, "A"))


@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("ahead", [1, 2, 4])
@pytest.mark.parametrize("inline,inline_max", [(8, 8), (24, 24), (8, 64)])
def test_fused_propose_seam_misses(parts, ahead, inline, inline_max):
    """A fused propose seam whose deltas overflow the inline part on some rank is applied
    nowhere (GC_H_SEAM); the host clears the halt and takes the unfused path.  Sweep seams
    run ahead of the host (``ahead``) halt the same way at the first overflow: the host
    moves that seam's deltas and runs the sweeps behind it again.  (8, 64): the inline part
    follows the frontiers, and a round whose frontier outgrew the last one's misses."""
    ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s1"))
    res = run_threads(rp, col, parts, inline=inline, inline_max=inline_max, deferred_ops=True, ahead=ahead)
    assert max(r.fused_misses for r in res) > 0
    for r in res:
        assert_matches_oracle(r, oracle.c_color(rp, col, "A"))


@pytest.mark.parametrize("ahead", [2, 4])
def test_sweep_seams_ahead_overflow(ahead):
    """Sweep seams run ahead of the host whose deltas overflow the inline part (the stand-in
    sends every sweep delta three times): the first such seam halts every rank, the host
    moves its deltas and runs the sweeps behind it again; the result is unchanged."""
    ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s1"))
    res = run_threads(rp, col, 2, inline=48, inline_max=48, shard_cls=InflatedShard, ahead=ahead)
    assert max(r.ahead_misses for r in res) > 0 and min(r.ahead_seams for r in res) > 0
    for r in res:
        assert_matches_oracle(r, oracle.c_color(rp, col, "A"))


@pytest.mark.parametrize("deferred_ops", [False, True])
@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("switch_below", [1, 40, 150, 10**9])
def test_hybrid_switch_to_one_engine(parts, switch_below, deferred_ops):
    """hybrid_color: the sharded rounds while the frontier is large, then the rest from the
    exported state on one engine (the stand-in for gc_color_resume): records, colours and
    rounds equal the single-partition oracle's for every switch point -- never (1), mid-run,
    and at round 0 (10**9) -- with the fused seams and the enqueue-only finish too."""
    for seed in range(3):
        rp, col = _random_directed(400, 2400, 30 + seed)
        o = oracle.c_color(rp, col, "A")
        calls = []
        res = run_threads(rp, col, parts, deferred_ops=deferred_ops, switch_below=switch_below, calls=calls)
        for r in res:
            assert_matches_oracle(r, o)
            assert r.switch_round == (calls[0][0] if calls else None)
        if switch_below == 1:
            assert not calls
        elif switch_below == 10**9:
            assert calls[0][0] == 0
        if calls:  # the frontier handed over is the one the oracle's switch round proposed on
            assert calls[0][1] == o["round_F"][calls[0][0]] and calls[0][1] < switch_below
    ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s1"))
    calls = []
    res = run_threads(rp, col, parts, deferred_ops=deferred_ops, switch_below=switch_below, calls=calls)
    assert_matches_oracle(res[-1], oracle.c_color(rp, col, "A"))


@pytest.mark.parametrize("seed", range(3))
def test_hybrid_bounded_stalled_and_reseeded(seed):
    """A bounded run that fails, a stall without E1 and E1 re-seeds on either side of the
    switch: the engine's records continue the sharded ones."""
    rp, col = _random_directed(300, 900, seed)
    o = oracle.c_color(rp, col, "A")
    for sw in (5, 30):
        assert_matches_oracle(run_threads(rp, col, 2, switch_below=sw, deferred_ops=True)[0], o)
        for k in (1, 2, int(o["max_color"])):
            assert_matches_oracle(run_threads(rp, col, 2, k=k, switch_below=sw)[1], oracle.c_color(rp, col, "A", k=k))
        s = oracle.c_color(rp, col, "A", e1=False)
        r = run_threads(rp, col, 3, e1=False, switch_below=sw)[0]
        assert r.status == s["status"] and np.array_equal(r.colors, s["colors"])
        assert list(r.round_U) == list(s["round_U"])


@pytest.mark.parametrize("case", ["single", "isolated3", "edge", "selfloop"])
def test_hybrid_tiny_graphs(case):
    """Tiny graphs (nothing to colour, one round, a self-loop) through the hybrid, with more ranks
    than vertices, switching never / at round 0."""
    rp, col = {"single": ([0, 0], []), "isolated3": ([0, 0, 0, 0], []), "edge": ([0, 1, 2], [1, 0]),
               "selfloop": ([0, 1], [0])}[case]
    rp, col = np.array(rp, np.int64), np.array(col, np.int32)
    o = oracle.c_color(rp, col, "A")
    for parts in (1, 3):
        for sw in (1, 10**9):
            for d in (False, True):
                for r in run_threads(rp, col, parts, switch_below=sw, deferred_ops=d):
                    assert_matches_oracle(r, o)


def test_more_ranks_than_vertices():
    rp = np.array([0, 1, 2], np.int64)
    col = np.array([1, 0], np.int32)
    res = run_threads(rp, col, 4)
    assert_matches_oracle(res[3], oracle.c_color(rp, col, "A"))


# ---- two processes over torch.distributed (gloo), the transport the GPU ranks use -------
def _gloo_worker(rank, world, port, path, out_dir, dense=None, inline=4096, deferred_ops=False, switch_below=None):
    import torch.distributed as dist
    sys.path[:0] = [PKG_DIR, REPO, os.path.dirname(os.path.abspath(__file__))]
    from shard_numpy import DeferredNumpyShard, NumpyShard, numpy_resume
    NS = DeferredNumpyShard if deferred_ops else NumpyShard
    from gcolor_amd import shard as shm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    d = np.load(path)
    rp, col = d["rp"], d["col"]
    lo, hi = shm.balanced_ranges(rp, world)[rank]
    kw = dict(track_rounds=True, dense=dense, inline=inline, inline_max=inline)
    if switch_below is None:
        res = shm.shard_color(NS(rp, col, lo, hi), shm.TorchTransport(), None, True, **kw)
    else:
        res = shm.hybrid_color(NS(rp, col, lo, hi), shm.TorchTransport(), numpy_resume(rp, col), switch_below, None,
                               True, **kw)
    out = {"status": res.status, "colors": res.colors.tolist(), "cround": res.colored_round.tolist(),
           "U": res.round_U, "F": res.round_F, "maxmex": res.round_maxmex, "acc": res.round_accepted,
           "seeds": res.round_seeds}
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("case,dense,inline,deferred_ops,switch_below", [
    ("gen_1000_8_s1", None, 4096, False, None), ("gen_1000_8_s1", True, 4096, False, None),
    ("asymmetric", None, 4096, False, None), ("gen_1000_8_s1", None, 3, False, None),
    ("gen_1000_8_s1", False, 0, False, None), ("gen_1000_8_s1", None, 4096, True, None),
    ("asymmetric", None, 3, True, None), ("gen_1000_8_s1", None, 4096, True, 60), ("asymmetric", None, 3, False, 4)])
def test_gloo_world_size_2(case, dense, inline, deferred_ops, switch_below, tmp_path):
    ids, adj, rp, col = fixture_csr(load_golden(case))
    path = str(tmp_path / "g.npz")
    np.savez(path, rp=rp, col=col)
    port = free_port()
    torch.multiprocessing.spawn(_gloo_worker,
                                args=(2, port, path, str(tmp_path), dense, inline, deferred_ops, switch_below),
                                nprocs=2, join=True)
    o = oracle.c_color(rp, col, "A")
    for r in range(2):
        got = json.load(open(tmp_path / f"r{r}.json"))
        assert got["status"] == o["status"]
        assert got["colors"] == list(o["colors"])
        assert got["cround"] == list(o["colored_round"])
        assert got["U"] == list(o["round_U"]) and got["F"] == list(o["round_F"])
        assert got["acc"] == list(o["round_accepted"]) and got["seeds"] == list(o["round_seeds"])


@pytest.mark.parametrize("parts", [1, 3])
def test_hybrid_switch_after_peak(parts):
    """switch_after_peak (the bench's hybrid): the switch waits until some round's frontier
    reached the switch point -- a first frontier below it (the seeds' neighbours) no longer
    ends the sharded rounds at round 0 -- or until SWITCH_GRACE rounds have run; records and
    colours equal the oracle's either way."""
    for seed in range(3):
        rp, col = _random_directed(400, 2400, 50 + seed)
        o = oracle.c_color(rp, col, "A")
        F = [int(x) for x in o["round_F"]]
        sw = max(F) // 2 + 1  # reached in some round, not in round 0 when the frontier grows first
        want = next((i for i, f in enumerate(F)
                     if 0 < f < sw and (max(F[:i + 1]) >= sw or i >= sh.SWITCH_GRACE)), None)
        calls = []
        res = run_threads(rp, col, parts, switch_below=sw, calls=calls, switch_after_peak=True)
        for r in res:
            assert_matches_oracle(r, o)
        assert (calls[0][0] if calls else None) == want
        calls = []  # a switch point no round reaches: after SWITCH_GRACE rounds
        res = run_threads(rp, col, parts, switch_below=10**9, calls=calls, switch_after_peak=True)
        for r in res:
            assert_matches_oracle(r, o)
        if len(F) > sh.SWITCH_GRACE and any(f > 0 for f in F[sh.SWITCH_GRACE:]):
            assert calls[0][0] == next(i for i, f in enumerate(F) if i >= sh.SWITCH_GRACE and f > 0)


@pytest.mark.parametrize("world,switch_below,deferred_ops", [(4, None, False), (4, 60, True), (8, 60, False)])
def test_gloo_more_ranks(world, switch_below, deferred_ops, tmp_path):
    """The driver's scaling runs use 4 and 8 ranks: the same exchange with 4 / 8 gloo processes
    (every round sharded, and the hybrid's hand-over), every rank bit-exact with the oracle."""
    ids, adj, rp, col = fixture_csr(load_golden("gen_1000_8_s1"))
    path = str(tmp_path / "g.npz")
    np.savez(path, rp=rp, col=col)
    port = free_port()
    torch.multiprocessing.spawn(_gloo_worker,
                                args=(world, port, path, str(tmp_path), None, 4096, deferred_ops, switch_below),
                                nprocs=world, join=True)
    o = oracle.c_color(rp, col, "A")
    for r in range(world):
        got = json.load(open(tmp_path / f"r{r}.json"))
        assert got["status"] == o["status"]
        assert got["colors"] == list(o["colors"])
        assert got["cround"] == list(o["colored_round"])
        assert got["U"] == list(o["round_U"]) and got["acc"] == list(o["round_accepted"])
