"""gc_color_resume, the multi-GPU hybrid and the closing commit's stage-overflow corner on the
GPU (promoted from tests/test_gpu_staged.py in round 4, after their first green run:
profiles/r04/a, profiles/r04/b).

* resume: gc_color_resume (include/gcolor.h) from the state at a round start, against the
  uninterrupted run -- records and colours -- and its rejection of an out-of-range frontier.
* hybrid: sharded rounds, then every rank's own one-GPU engine (gcolor_amd.shard.hybrid_color),
  on threads and as two processes over torch.distributed, against one GPU.
* overflow_tree / under_ticket_close: a closing commit (arrival tickets on the next frontier's
  counter) whose waves overflow their LDS stage mid-launch -- round 3's k_commit aperture fault
  (DESIGN §5): the flush base masked (GC_COUNT_MASK) and bounded by the list capacity.
* validate_c8: gc_validate of the resident colouring from the byte mirror c8 (the default since
  round 4) against the int colours and the oracle's validator (coloring.py:149-162).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402,F401

pytestmark = pytest.mark.gpu


# --- gc_color_resume and the multi-GPU hybrid -----------------------------------------------
import test_shard_gpu as sg  # noqa: E402


def _state_at(rp, col, colors, cround, r):
    """the engine's state at the start of round r, from an uninterrupted run's colours and
    rounds (coloured in round q -> cround q + 1; the seed and isolated vertices -> 0): the
    colours so far and the frontier (uncoloured, with a coloured listed neighbour)."""
    c = np.where(cround <= r, colors, -1).astype(np.int32)
    cr = np.where(cround <= r, cround, -1).astype(np.int32)
    deg = np.diff(rp)
    src = np.repeat(np.arange(len(deg)), deg)
    has = np.zeros(len(deg), bool)
    np.logical_or.at(has, src, c[col] >= 0)
    front = np.nonzero((c < 0) & has)[0].astype(np.int32)
    return c, cr, front


def _resume_matches(dg, rounds_at):
    import torch
    one = dg.color("A")
    rp, col = dg.export()
    for r in rounds_at:
        r = min(r, one.rounds - 1)
        c, cr, front = _state_at(rp, col, one.colors, one.colored_round, r)
        ct, crt, ft = (torch.from_numpy(x).cuda() for x in (c, cr, front if len(front) else np.zeros(1, np.int32)))
        torch.cuda.synchronize()
        g = dg.resume(ct.data_ptr(), ft.data_ptr(), len(front), r, cround_dev=crt.data_ptr())
        assert g.status == one.status
        assert np.array_equal(g.colors, one.colors) and np.array_equal(g.colored_round, one.colored_round)
        for k in ("round_U", "round_F", "round_maxmex", "round_accepted", "round_seeds"):
            assert list(getattr(g, k)) == list(getattr(one, k))[r:], (k, r)


def test_resume_golden_and_directed():
    from gcolor_amd.engine import DeviceGraph
    for name in sg.GOLD[::4]:
        ids, adj, rp, col = sg.fixture_csr(sg.load_golden(name))
        with DeviceGraph.from_csr(rp, col) as dg:
            _resume_matches(dg, [0, 1, 3, 10**9])
    for seed in range(2):
        rp, col = sg._random_directed(3000, 9000, seed)
        with DeviceGraph.from_csr(rp, col) as dg:
            _resume_matches(dg, [0, 2, 7, 10**9])


@pytest.mark.parametrize("scale", [10, 14])
def test_resume_rmat_hubs(scale):
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(scale, 16, seed=2) as dg:
        _resume_matches(dg, [0, 5, 40, 200])


@pytest.mark.parametrize("switch_below", [1, 64, 2048, 10**9])
def test_hybrid_threads(switch_below):
    from gcolor_amd.engine import DeviceGraph
    for name in sg.GOLD[::5]:
        ids, adj, rp, col = sg.fixture_csr(sg.load_golden(name))
        with DeviceGraph.from_csr(rp, col) as dg:
            sg.same_as_single(dg, 3, switch_below=switch_below)
    rp, col = sg._random_directed(3000, 9000, 1)
    with DeviceGraph.from_csr(rp, col) as dg:
        r, one = sg.same_as_single(dg, 2, switch_below=switch_below)
        sg.same_as_single(dg, 3, k=max(one.max_color, 1), switch_below=switch_below)
        sg.same_as_single(dg, 2, e1=False, switch_below=switch_below)
    with DeviceGraph.rmat(13, 16, seed=4) as dg:
        r, _ = sg.same_as_single(dg, 4, switch_below=switch_below)
        assert (r.switch_round is None) == (switch_below == 1)



@pytest.mark.parametrize("env", [{}, {"GC_FUSE": "0"}], ids=["fused", "unfused"])
def test_commit_stage_overflow_under_ticket_close(env, monkeypatch):
    """tests/commit_cases.py: 32768 winners in the first 2048 wave chunks of a 16M-vertex graph
    (frontier < n/256: the commit closes its own round with arrival tickets), each claiming 40
    leaves -- 640 pushes per busy wave, past the 512-entry stage, after the 1024 idle waves have
    taken their tickets.  Round 3's build took the mid-launch flush's base from the ticketed
    counter (the 10M uniform fault); the colours and records must be exact."""
    import torch
    from commit_cases import stage_overflow_case
    from gcolor_amd.engine import DeviceGraph
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rp, col, c, front, exp = stage_overflow_case(32768, 40, 1 << 24)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        ct, ft = torch.from_numpy(c).cuda(), torch.from_numpy(front).cuda()
        torch.cuda.synchronize()
        g = dg.resume(ct.data_ptr(), ft.data_ptr(), len(front), 5)
        assert g.status == 0
        assert list(g.round_F[:2]) == exp["F"] and list(g.round_accepted[:2]) == exp["accepted"]
        assert list(g.round_U[:2]) == exp["U"]
        assert np.array_equal(g.colors, exp["colors"])
        assert dg.validate() == (0, 0)


@pytest.mark.parametrize("env", [{}, {"GC_FUSE": "0"}], ids=["fused", "unfused"])
def test_commit_stage_overflow_tree(env, monkeypatch):
    """The same corner from a plain colouring (no resume; tests/commit_cases.py): a fanout-61
    tree padded to 2^26 vertices.  Round 2's frontier is its 234,423 level-3 vertices (< n/256:
    a closing commit), 128 per busy wave x 61 claimed children = 7,808 pushes (15 mid-launch
    flushes), while the 1,240 waves without a chunk take their tickets at once.  Candidate for
    the default GPU suite once green (it runs the default path only)."""
    from commit_cases import stage_overflow_tree
    from gcolor_amd.engine import DeviceGraph
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rp, col, exp = stage_overflow_tree(61, 5, 1 << 26)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("A")
        assert g.status == 0
        assert list(g.round_F[:-1]) == exp["F"] and list(g.round_accepted[:-1]) == exp["F"]
        assert np.array_equal(g.colors, exp["colors"])
        assert dg.validate() == (0, 0)


def test_resume_rejects_out_of_range_frontier():
    """A frontier entry outside [0, n) stops gc_color_resume before any round (GC_EINVAL)."""
    import torch
    from gcolor_amd import _native as nat
    from gcolor_amd.engine import DeviceGraph
    rp, col = sg._random_directed(500, 2000, 3)
    with DeviceGraph.from_csr(rp, col) as dg:
        c = torch.full((dg.n,), -1, dtype=torch.int32, device="cuda")
        c[0] = 0
        f = torch.tensor([1, dg.n + 7], dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        with pytest.raises(nat.GcolorError, match="out of range"):
            dg.resume(c.data_ptr(), f.data_ptr(), 2, 0)
        assert dg.color("A").status == 0  # the handle is still usable


def _hybrid_gpu_worker(rank, world, port, out_dir):
    import json
    import torch
    import torch.distributed as dist
    sys.path[:0] = [sg.PKG_DIR, sg.REPO]
    torch.cuda.set_device(0)
    from gcolor_amd.engine import DeviceGraph
    from gcolor_amd import shard as sh
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    out = {}
    with DeviceGraph.rmat(12, 16, seed=9) as dg:
        rp, _ = dg.export(col=False)
        lo, hi = sh.balanced_ranges(rp, world)[rank]
        ops = sh.HipShard(dg, lo, hi)
        for sw in (256, 10**9):
            res = sh.hybrid_color(ops, sh.TorchTransport(), sh.engine_resume(dg), sw, track_rounds=True)
            out[str(sw)] = {"colors": res.colors.tolist(), "cround": res.colored_round.tolist(), "U": res.round_U,
                            "acc": res.round_accepted, "switch": res.switch_round}
        ops.close()
    with open(os.path.join(out_dir, f"h{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


def test_hybrid_two_processes(tmp_path):
    """The hybrid as two processes over torch.distributed (gloo; both ranks on the one GPU):
    sharded rounds, the frontier parts all-gathered, each rank resuming its own engine."""
    import json
    import torch
    from conftest import free_port
    from gcolor_amd.engine import DeviceGraph
    port = free_port()
    torch.multiprocessing.spawn(_hybrid_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    with DeviceGraph.rmat(12, 16, seed=9) as dg:
        one = dg.color("A")
    for r in range(2):
        got = json.load(open(tmp_path / f"h{r}.json"))
        for sw, res in got.items():
            assert res["colors"] == list(one.colors) and res["cround"] == list(one.colored_round), sw
            assert res["U"] == list(one.round_U) and res["acc"] == list(one.round_accepted), sw
        assert got["1000000000"]["switch"] == 0


# --- validation of the resident colouring from the byte mirror (default since round 4) ---------
def test_validate_c8_matches(monkeypatch):
    """The resident colouring validated from c8 (the default since round 4; GC_VALIDATE_C8=0
    gathers the int colours) counts what the int colours count: after a full
    run, after a failed bounded run (uncoloured vertices), and after a resume from a state with
    planted conflicts (colours < 254 and >= 254, the byte mirror's BIG case)."""
    import torch
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(12, 16, seed=9) as dg:
        rp, col = dg.export()
        for k in (None, 3):
            g = dg.color("A", num_colors=k)
            monkeypatch.setenv("GC_VALIDATE_C8", "0")
            ref = dg.validate()
            monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
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
        monkeypatch.setenv("GC_VALIDATE_C8", "0")
        ref = dg.validate()
        monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
        assert dg.validate() == ref == tuple(oracle.c_validate(rp, col, g.colors))
        assert ref[1] > 0



@pytest.mark.parametrize("half", ["1", "0"], ids=["low_parts", "every_entry"])
def test_validate_symmetric_half(monkeypatch, half):
    """gc_validate of a symmetric graph reads only the low parts of the rank partition and counts
    2 x their conflicts + the self-loop entries (round 4; GC_VALIDATE_HALF=0 reads every entry):
    equal to the oracle's directed count (coloring.py:149-162) on a symmetric multigraph with
    duplicates, self-loops and a row past the tile height (its segments), under arbitrary colour
    arrays (uncoloured, colours < 254 and >= 254) and after real colourings."""
    from gcolor_amd.engine import DeviceGraph
    monkeypatch.setenv("GC_VALIDATE_HALF", half)
    rng = np.random.default_rng(11)
    n = 6000
    a = rng.integers(0, n, 40000)
    b = rng.integers(0, n, 40000)
    a = np.concatenate([a, np.zeros(3000, np.int64), a[:500]])  # vertex 0 a row of > 3000 entries; duplicates
    b = np.concatenate([b, rng.integers(1, n, 3000), b[:500]])
    keep = a != b
    src = np.concatenate([a[keep], b[keep], np.arange(0, n, 97)])  # self-loops: one entry each
    dst = np.concatenate([b[keep], a[keep], np.arange(0, n, 97)])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    rp = np.cumsum(rp)
    col = dst.astype(np.int32)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("A")
        assert tuple(dg.validate()) == tuple(oracle.c_validate(rp, col, g.colors))
        g = dg.color("A", num_colors=2)  # failed: uncoloured vertices
        assert tuple(dg.validate()) == tuple(oracle.c_validate(rp, col, g.colors))
        for palette in (3, 400):
            c = rng.integers(-1, palette, n).astype(np.int32)
            assert tuple(dg.validate(c)) == tuple(oracle.c_validate(rp, col, c))


def _sym_multigraph(seed, n=6000):
    """The multigraph of test_validate_symmetric_half: duplicates, self-loops, a > 3000-entry row."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n, 40000)
    b = rng.integers(0, n, 40000)
    a = np.concatenate([a, np.zeros(3000, np.int64), a[:500]])
    b = np.concatenate([b, rng.integers(1, n, 3000), b[:500]])
    keep = a != b
    src = np.concatenate([a[keep], b[keep], np.arange(0, n, 97)])
    dst = np.concatenate([b[keep], a[keep], np.arange(0, n, 97)])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


def _range_counts(rp, col, colors, lo, hi, half):
    """gc_validate_range's counts restated in numpy: rows [lo, hi) of the directed count
    (coloring.py:149-162), or -- symmetric graphs, low parts only -- 2 x the conflicts of the
    rows' lower-rank entries (rank (deg, pos), coloring.py:64) + their self-loop entries."""
    n = len(rp) - 1
    deg = np.diff(rp)
    e0, e1 = int(rp[lo]), int(rp[hi])
    rows = np.repeat(np.arange(lo, hi), deg[lo:hi])
    u = col[e0:e1].astype(np.int64)
    same = colors[u] == colors[rows]
    unc = int(np.count_nonzero(colors[lo:hi] == -1))
    if not half:
        return unc, int(np.count_nonzero(same))
    key = deg.astype(np.int64) * n + np.arange(n)
    low = key[u] < key[rows]
    return unc, int(2 * np.count_nonzero(same & low) + np.count_nonzero(u == rows))


@pytest.mark.parametrize("half", ["1", "0"], ids=["low_parts", "every_entry"])
def test_validate_range(monkeypatch, half):
    """gc_validate_range (the multi-GPU step's split of validate_graph_coloring, coloring.py:149-162):
    each range's counts equal the numpy restatement of the rows it holds -- ranges cut inside tiles,
    around the segmented > 3000-entry row of vertex 0, single vertices, empty -- and any cover of
    [0, n) by disjoint ranges adds up to the oracle's counts, for the resident colouring and for
    arbitrary colour arrays."""
    from gcolor_amd.engine import DeviceGraph
    monkeypatch.setenv("GC_VALIDATE_HALF", half)
    rp, col = _sym_multigraph(12)
    n = len(rp) - 1
    rng = np.random.default_rng(5)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        g = dg.color("A")
        arrays = [None, rng.integers(-1, 3, n).astype(np.int32), rng.integers(-1, 400, n).astype(np.int32)]
        for c in arrays:
            cc = g.colors if c is None else c
            full = oracle.c_validate(rp, col, cc)
            for cuts in ([0, 1, n], [0, 2, 3, 4000, n], sorted(set([0, n] + list(rng.integers(0, n, 7)))), [0, n // 2, n]):
                tot = np.zeros(2, np.int64)
                for lo, hi in zip(cuts[:-1], cuts[1:]):
                    got = dg.validate(c, lo=lo, hi=hi)
                    assert tuple(got) == _range_counts(rp, col, cc, lo, hi, half == "1"), (lo, hi)
                    tot += got
                assert tuple(tot) == tuple(full)
            assert dg.validate(c, lo=17, hi=17) == (0, 0)
        with pytest.raises(Exception):
            dg.validate(None, lo=-1, hi=5)
        with pytest.raises(Exception):
            dg.validate(None, lo=5, hi=n + 1)


@pytest.mark.parametrize("variant", ["A", "B"])
def test_list_overflow_reported_and_halted(monkeypatch, variant):
    """A staged list append that would pass its list's capacity writes nothing, halts the
    pipeline (every later kernel returns at once instead of reading the list up to the
    overflowed count) and comes back as GC_EHIP -- not a fault.  The capacity is
    lowered to 16 entries (GC_TEST_LIST_CAP; the buffers keep n entries, so a kernel that read
    past the logical end would still stay inside them); afterwards the same handle colours the
    graph exactly again."""
    from gcolor_amd import _native as nat
    from gcolor_amd.engine import DeviceGraph, uniform_csr
    rp, col = uniform_csr(200_000, 16, 3)
    with DeviceGraph.from_csr(rp, col, symmetric=True) as dg:
        ref = dg.color(variant)
        monkeypatch.setenv("GC_TEST_LIST_CAP", "16")
        with pytest.raises(nat.GcolorError) as ei:
            dg.color(variant)
        assert ei.value.status == nat.GC_EHIP and "capacity" in str(ei.value)
        monkeypatch.delenv("GC_TEST_LIST_CAP")
        again = dg.color(variant)
        assert np.array_equal(again.colors, ref.colors) and list(again.round_U) == list(ref.round_U)
    with DeviceGraph.rmat(16, 16, seed=2) as dg:  # hubs: the asynchronous JP / fold paths
        ref = dg.color(variant)
        monkeypatch.setenv("GC_TEST_LIST_CAP", "16")
        with pytest.raises(nat.GcolorError) as ei:
            dg.color(variant)
        assert ei.value.status == nat.GC_EHIP
        monkeypatch.delenv("GC_TEST_LIST_CAP")
        assert np.array_equal(dg.color(variant).colors, ref.colors)
