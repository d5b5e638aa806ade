"""Multi-GPU colouring: vertex-range shards, one rank per GPU.

Every rank holds the whole CSR (a ``DeviceGraph``) and owns a contiguous, nnz-balanced
range of vertices.  A round is the single-GPU round (coloring.py:73-132) cut at its three
grid-wide seams.  At each seam every rank publishes what changed on its own vertices,
as int64 deltas ``vertex << 32 | value``, and applies everyone else's:

    propose               (v, candidate)   all-gather -> apply     coloring.py:44-54
    first sweep, sweeps   (v, IN | OUT)    all-gather -> apply     coloring.py:56-70
    accept                (v, colour)      all-gather -> push      coloring.py:114-127

The round scalars (frontier size, max proposal, failures, undecided, accepted) travel in a
small all-gather next to each delta all-gather.  Conflict resolution is the
lexicographically-first MIS under the global rank (deg, pos), so the colouring does not
depend on the partition: it is bit-identical to one GPU.  E1 re-seeding runs on every
rank over the replicated state, so every rank plants the same seeds.

``shard_color(ops, comm)`` is the SPMD driver.
* ``ops`` is one rank's phase implementation: ``HipShard`` here (libgcolor.so); the
  CPU stand-in used by the ``gloo`` tests lives in ``tests/``.
* ``comm`` moves the deltas: ``TorchTransport`` (torch.distributed; RCCL over xGMI with
  ``nccl``, or ``gloo``), or ``ThreadTransport`` for several shards in one process.
"""
import threading
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat

KIND_CAND, KIND_STATE, KIND_COLOUR = 0, 1, 2
OK, FAILED, STALLED = 0, 1, 2


def balanced_ranges(rp, parts):
    """Contiguous vertex ranges with about equal (deg + 1) weight, one per rank."""
    rp = np.asarray(rp, dtype=np.int64)
    n = rp.shape[0] - 1
    w = rp + np.arange(n + 1, dtype=np.int64)  # prefix sums of (deg + 1)
    targets = (w[-1] * np.arange(parts + 1, dtype=np.int64)) // parts
    b = np.searchsorted(w, targets, side="left")
    b[0], b[-1] = 0, n
    b = np.maximum.accumulate(np.minimum(b, n))
    return [(int(b[i]), int(b[i + 1])) for i in range(parts)]


# ------------------------------------------------------------------------------------------
# transports
# ------------------------------------------------------------------------------------------
class TorchTransport:
    """All-gather over a torch.distributed group: RCCL (``nccl``) on device tensors, or
    ``gloo`` (device tensors are staged through host memory)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = str(dist.get_backend(group))

    def _allgather(self, out, inp):
        if self.backend == "nccl":
            self.dist.all_gather_into_tensor(out, inp, group=self.group)
        else:
            self.dist.all_gather(list(out.chunk(self.size)), inp, group=self.group)

    def exchange(self, stats, delta, count):
        """stats: ints of this rank; delta[:count]: its deltas.  Returns (all ranks' stats
        as an int64 array [size, len(stats) + 1] whose last column is the counts, the
        concatenated deltas padded with -1 entries (or None), its length)."""
        dev = delta.device if delta is not None else torch.device("cpu")
        cdev = dev if self.backend == "nccl" else torch.device("cpu")
        s = torch.tensor(list(stats) + [int(count)], dtype=torch.int64, device=cdev)
        all_s = torch.empty(self.size * s.numel(), dtype=torch.int64, device=cdev)
        self._allgather(all_s, s)
        all_s = all_s.view(self.size, -1).cpu().numpy()
        maxc = int(all_s[:, -1].max())
        if maxc == 0:
            return all_s, None, 0
        send = torch.full((maxc,), -1, dtype=torch.int64, device=cdev)
        if count:
            send[:count].copy_(delta[:count])
        recv = torch.empty(self.size * maxc, dtype=torch.int64, device=cdev)
        self._allgather(recv, send)
        if recv.device != dev:
            recv = recv.to(dev)
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()
        return all_s, recv, int(recv.numel())


class ThreadHub:
    """Rendezvous for ``parts`` shards driven by threads of one process."""

    def __init__(self, parts):
        self.parts = parts
        self.barrier = threading.Barrier(parts)
        self.box = [None] * parts


class ThreadTransport:
    def __init__(self, hub, rank):
        self.hub, self.rank, self.size = hub, rank, hub.parts

    def exchange(self, stats, delta, count):
        h = self.hub
        part = delta[:count].clone() if count else None
        if part is not None and part.is_cuda:
            torch.cuda.current_stream(part.device).synchronize()
        h.box[self.rank] = (list(stats) + [int(count)], part)
        h.barrier.wait()
        all_s = np.array([b[0] for b in h.box], dtype=np.int64)
        parts = [b[1] for b in h.box if b[1] is not None]
        recv = torch.cat(parts) if parts else None
        if recv is not None and recv.is_cuda:
            torch.cuda.current_stream(recv.device).synchronize()
        h.barrier.wait()  # every rank has copied the box before it is refilled
        return all_s, recv, 0 if recv is None else int(recv.numel())


# ------------------------------------------------------------------------------------------
# HIP phase implementation (libgcolor.so)
# ------------------------------------------------------------------------------------------
def _p(t):
    return None if t is None else t.data_ptr()


class HipShard:
    """One rank's share on its GPU: ``gc_shard_*`` of libgcolor.so."""

    def __init__(self, dg, lo, hi, device=None):
        import ctypes
        self._ct = ctypes
        self._lib = nat.load()
        self.dg, self.lo, self.hi, self.n = dg, int(lo), int(hi), dg.n
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        h = ctypes.c_void_p()
        nat.check("gc_shard_create", self._lib.gc_shard_create(dg._h, self.lo, self.hi, ctypes.byref(h)))
        self._h = h
        self.cap = max(self.hi - self.lo, 1)
        self.delta = torch.empty(self.cap, dtype=torch.int64, device=self.device)
        self._st = (ctypes.c_int64 * 4)()
        self._a = ctypes.c_int64()
        self._b = ctypes.c_int64()

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gc_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def begin(self, k, track_rounds):
        ct = self._ct
        nat.check("gc_shard_begin", self._lib.gc_shard_begin(self._h, int(k), 1 if track_rounds else 0,
                                                             ct.byref(self._a), ct.byref(self._b)))
        return self._a.value, self._b.value

    def propose(self, r):
        nat.check("gc_shard_propose", self._lib.gc_shard_propose(self._h, r, _p(self.delta), self.cap, self._st))
        return self._st[0], self._st[1], self._st[2], self._st[3]

    def apply(self, kind, recv, count, r):
        if count:
            nat.check("gc_shard_apply", self._lib.gc_shard_apply(self._h, kind, _p(recv), count, r))

    def sweep(self, i):
        nat.check("gc_shard_sweep", self._lib.gc_shard_sweep(self._h, i, _p(self.delta), self.cap, self._st))
        return self._st[0], self._st[1]

    def accept(self, r):
        nat.check("gc_shard_accept", self._lib.gc_shard_accept(self._h, r, _p(self.delta), self.cap, self._st))
        return self._st[0]

    def push(self, r, recv, count):
        nat.check("gc_shard_push", self._lib.gc_shard_push(self._h, r, _p(recv), count, self._ct.byref(self._a)))
        return self._a.value

    def reseed(self, r):
        ct = self._ct
        nat.check("gc_shard_reseed", self._lib.gc_shard_reseed(self._h, r, ct.byref(self._a), ct.byref(self._b)))
        return self._a.value, self._b.value

    def colors(self, track_rounds):
        colors = np.empty(self.n, np.int32)
        cround = np.empty(self.n, np.int32) if track_rounds else None
        nat.check("gc_shard_colors", self._lib.gc_shard_colors(
            self._h, colors.ctypes.data_as(self._ct.c_void_p),
            None if cround is None else cround.ctypes.data_as(self._ct.c_void_p)))
        return colors, cround


# ------------------------------------------------------------------------------------------
# the SPMD driver
# ------------------------------------------------------------------------------------------
@dataclass
class ShardResult:
    status: int
    colors: np.ndarray
    colored_round: np.ndarray
    round_U: list = field(default_factory=list)
    round_F: list = field(default_factory=list)
    round_maxmex: list = field(default_factory=list)
    round_accepted: list = field(default_factory=list)
    round_seeds: list = field(default_factory=list)
    fail_round: int = -1
    fail_count: int = 0
    reseeds: int = 0
    jp_sweeps: int = 0
    exchanges: int = 0

    @property
    def rounds(self):
        return len(self.round_U)

    @property
    def max_color(self):
        return int(self.colors.max()) if len(self.colors) else -1


def shard_color(ops, comm, num_colors=None, e1=True, track_rounds=False):
    """graph_coloring (coloring.py:73) over the ranks of ``comm``; every rank returns the
    same ShardResult (records with the single-GPU semantics of gc_color)."""
    k = -1 if num_colors is None else int(num_colors)
    U, _ = ops.begin(k, track_rounds)
    res = ShardResult(status=OK, colors=None, colored_round=None)

    def rec(u, f, mm, acc, seeds):
        res.round_U.append(int(u))
        res.round_F.append(int(f))
        res.round_maxmex.append(int(mm))
        res.round_accepted.append(int(acc))
        res.round_seeds.append(int(seeds))

    def xchg(stats, count):
        res.exchanges += 1
        return comm.exchange(stats, ops.delta, count)

    max_rounds = 4 * ops.n + 16
    r = 0
    while True:
        if U == 0:  # coloring.py:86-90
            rec(0, 0, -1, 0, 0)
            break
        if r > max_rounds:
            raise RuntimeError("round limit exceeded")
        cnt, f_loc, mm, fails = ops.propose(r)
        S, recv, tot = xchg([f_loc, mm, fails], cnt)
        F, maxmex, fails = int(S[:, 0].sum()), int(S[:, 1].max()), int(S[:, 2].sum())
        if F == 0:  # no proposer anywhere: the reference spins (coloring.py:93-95) -> E1
            if not e1:
                rec(U, 0, -1, 0, 0)
                res.status = STALLED
                break
            ns, _ = ops.reseed(r)
            rec(U, 0, -1, 0, ns)
            res.reseeds += ns
            U -= ns
            r += 1
            continue
        if k >= 0 and fails > 0:  # coloring.py:104-108
            rec(U, F, maxmex, 0, 0)
            res.status, res.fail_round, res.fail_count = FAILED, r, fails
            break
        ops.apply(KIND_CAND, recv, tot, r)
        cnt, und = ops.sweep(0)
        S, recv, tot = xchg([und], cnt)
        ops.apply(KIND_STATE, recv, tot, r)
        und, i = int(S[:, 0].sum()), 1
        while und > 0:
            cnt, und = ops.sweep(i)
            S, recv, tot = xchg([und], cnt)
            ops.apply(KIND_STATE, recv, tot, r)
            und, i = int(S[:, 0].sum()), i + 1
            res.jp_sweeps += 1
        cnt = ops.accept(r)
        S, recv, tot = xchg([], cnt)
        acc = int(S[:, -1].sum())
        ops.push(r, recv, tot)
        rec(U, F, maxmex, acc, 0)
        U -= acc
        r += 1
    res.colors, res.colored_round = ops.colors(track_rounds)
    return res


def color_threads(dg, parts, num_colors=None, e1=True, track_rounds=False):
    """``parts`` shards of one colouring on the current GPU, driven by threads: the test
    and rehearsal path of the multi-GPU engine on one device."""
    rp, _ = dg.export()
    ranges = balanced_ranges(rp, parts)
    hub = ThreadHub(parts)
    # the CSR is read-only: every shard borrows it, each keeps its own replicated state
    shards = [HipShard(dg, lo, hi) for lo, hi in ranges]
    out = [None] * parts
    err = []

    def run(i):
        try:
            out[i] = shard_color(shards[i], ThreadTransport(hub, i), num_colors, e1, track_rounds)
        except BaseException as e:  # noqa: BLE001 - surface the first failure
            err.append(e)
            hub.barrier.abort()

    ts = [threading.Thread(target=run, args=(i,)) for i in range(parts)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for sh in shards:
        sh.close()
    if err:
        raise err[0]
    return out
