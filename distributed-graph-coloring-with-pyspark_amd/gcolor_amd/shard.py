"""Multi-GPU colouring: vertex-range shards, one rank per GPU.

Every rank holds the whole CSR (a ``DeviceGraph``) and owns a contiguous, nnz-balanced
range of vertices.  A round is the single-GPU round (coloring.py:73-132) cut at its
grid-wide seams.  At each seam every rank publishes what changed on its own vertices and
takes everyone else's:

    propose               (v, candidate)   all-gather -> apply     coloring.py:44-54
    first sweep, sweeps   (v, IN | OUT)    all-gather -> apply     coloring.py:56-70

as int64 deltas ``vertex << 32 | value`` -- or, when the padded deltas would outweigh
it, as every rank's slice of the proposal bytes (cand6 << 2 | state), copied back in
place.  After the last sweep seam every rank holds every proposer's final state, so each
colours ALL the round's winners itself (coloring.py:114-127) and pushes them into its own
in-neighbours: no exchange at commit.  The round scalars (frontier size, max proposal,
failures, undecided) travel as a header in front of each seam's payload, so a seam is
one all-gather unless some rank's deltas overflow the inline part.  When every seam of a
round moved deltas, the other ranks' winners are the IN states received, and the round
ends in O(winners); after a dense (slice) seam it scans the replicated proposal bytes.
Conflict resolution is the lexicographically-first MIS under the global rank (deg, pos),
so the colouring does not depend on the partition: it is bit-identical to one GPU.  E1
re-seeding runs on every rank over the replicated state, so every rank plants the same
seeds.

``shard_color(ops, comm)`` is the SPMD driver.
* ``ops`` is one rank's phase implementation: ``HipShard`` here (libgcolor.so); the
  CPU stand-in used by the ``gloo`` tests lives in ``tests/``.
* ``comm`` moves the data: ``TorchTransport`` (torch.distributed; RCCL over xGMI with
  ``nccl``, or ``gloo``), or ``ThreadTransport`` for several shards in one process.
"""
import threading
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat

KIND_CAND, KIND_STATE, KIND_COLOUR = 0, 1, 2
OK, FAILED, STALLED = 0, 1, 2
# hybrid: rounds after which the switch no longer waits for the frontier to reach the
# switch point (a graph whose frontier never gets that large)
SWITCH_GRACE = 8


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
    """All-gathers over a torch.distributed group: RCCL (``nccl``) on device tensors, or
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

    def _cdev(self, dev):
        return dev if self.backend == "nccl" else torch.device("cpu")

    def gather_stats(self, stats, device):
        """ints of this rank -> int64 array [size, len(stats)] of every rank's."""
        cdev = self._cdev(device)
        s = torch.tensor([int(x) for x in stats], dtype=torch.int64, device=cdev)
        out = torch.empty(self.size * s.numel(), dtype=torch.int64, device=cdev)
        self._allgather(out, s)
        return out.view(self.size, -1).cpu().numpy()

    def _gather_padded(self, send, dev):
        recv = torch.empty(self.size * send.numel(), dtype=send.dtype, device=send.device)
        self._allgather(recv, send)
        if recv.device != dev:
            recv = recv.to(dev)
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()
        return recv

    def gather_deltas(self, delta, count, maxc):
        """delta[:count] of every rank, each padded to maxc with -1 entries."""
        dev = delta.device
        send = torch.full((maxc,), -1, dtype=torch.int64, device=self._cdev(dev))
        if count:
            send[:count].copy_(delta[:count])
        return self._gather_padded(send, dev)

    def gather_slices(self, buf):
        """buf (uint8, the same length on every rank) of every rank, concatenated."""
        dev = buf.device
        send = buf if self._cdev(dev) == dev else buf.to(self._cdev(dev))
        return self._gather_padded(send, dev)

    def allgather(self, t):
        """t (1-D, the same length on every rank) of every rank, concatenated, on t's
        device.  With RCCL it is enqueued on the current stream: no host wait."""
        dev = t.device
        send = t if self._cdev(dev) == dev else t.to(self._cdev(dev))
        recv = torch.empty(self.size * send.numel(), dtype=send.dtype, device=send.device)
        self._allgather(recv, send)
        return recv if recv.device == dev else recv.to(dev)


class ThreadHub:
    """Rendezvous for ``parts`` shards driven by threads of one process."""

    def __init__(self, parts):
        self.parts = parts
        self.barrier = threading.Barrier(parts)
        self.box = [None] * parts


class ThreadTransport:
    def __init__(self, hub, rank):
        self.hub, self.rank, self.size = hub, rank, hub.parts

    def _gather(self, item):
        h = self.hub
        h.box[self.rank] = item
        h.barrier.wait()
        got = list(h.box)
        h.barrier.wait()  # every rank has read the box before it is refilled
        return got

    @staticmethod
    def _settle(t):
        if t is not None and t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()
        return t

    def gather_stats(self, stats, device):
        return np.array(self._gather([int(x) for x in stats]), dtype=np.int64)

    def gather_deltas(self, delta, count, maxc):
        part = torch.full((maxc,), -1, dtype=torch.int64, device=delta.device)
        if count:
            part[:count].copy_(delta[:count])
        self._settle(part)
        return self._settle(torch.cat(self._gather(part)))

    def gather_slices(self, buf):
        part = self._settle(buf.clone())
        return self._settle(torch.cat(self._gather(part)))

    def allgather(self, t):
        return self._settle(torch.cat(self._gather(self._settle(t.clone()))))


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
        # the shard's kernels run on the graph's device, so its stream and buffers live there
        self.device = torch.device("cuda", dg.device_index) if device is None else torch.device(device)
        if self.device.type != "cuda" or self.device.index not in (None, dg.device_index):
            raise ValueError(f"HipShard on {self.device}: the graph lives on cuda:{dg.device_index}")
        if self.device.index is None:
            self.device = torch.device("cuda", dg.device_index)
        h = ctypes.c_void_p()
        nat.check("gc_shard_create", self._lib.gc_shard_create(dg._h, self.lo, self.hi, ctypes.byref(h)))
        self._h = h
        # the shard's kernels run on torch's current stream, where the collectives run
        if self.device.type == "cuda":
            nat.check("gc_shard_set_stream", self._lib.gc_shard_set_stream(
                h, ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        self.cap = max(self.hi - self.lo, 1)
        self.delta = torch.empty(self.cap, dtype=torch.int64, device=self.device)
        self._slice = None
        self._bufs = {}
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

    # ---- seams: the phase, then its send buffer built on the device (no host round trip) --
    def _send(self, n, dtype):
        key = (n, dtype)
        if key not in self._bufs:
            self._bufs[key] = torch.empty(n, dtype=dtype, device=self.device)
        return self._bufs[key]

    def propose_seam(self, r, C):
        """propose (enqueued) + send buffer: HDR header words and up to C deltas."""
        lib = self._lib
        nat.check("gc_shard_propose_async", lib.gc_shard_propose_async(self._h, r, _p(self.delta), self.cap))
        send = self._send(HDR + C, torch.int64)
        nat.check("gc_shard_pack", lib.gc_shard_pack(self._h, KIND_CAND, 0, _p(self.delta), _p(send), C))
        return send

    def sweep_seam(self, i, count, C, emit, stride):
        """JP sweeps i .. i+count-1 (enqueued) + send buffer: HDR header words and up to C
        deltas, or (emit=False, a slice seam) the header bytes and the rank's proposal-byte
        slice (stride bytes)."""
        lib = self._lib
        nat.check("gc_shard_sweep_async", lib.gc_shard_sweep_async(self._h, i, count, _p(self.delta) if emit else None,
                                                                   self.cap))
        last = (i + count - 1) % 3
        if emit:
            send = self._send(HDR + C, torch.int64)
            nat.check("gc_shard_pack", lib.gc_shard_pack(self._h, KIND_STATE, last, _p(self.delta), _p(send), C))
            return send
        buf = self._send(8 * HDR + stride, torch.uint8)
        nat.check("gc_shard_pack", lib.gc_shard_pack(self._h, KIND_STATE, last, None, _p(buf), 0))
        nat.check("gc_shard_get_slice", lib.gc_shard_get_slice(self._h, _p(buf[8 * HDR:])))
        return buf

    def apply(self, kind, recv, count, r):
        if count:
            nat.check("gc_shard_apply", self._lib.gc_shard_apply(self._h, kind, _p(recv), count, r))

    def sweep(self, i, count=1, emit=True):
        nat.check("gc_shard_sweep", self._lib.gc_shard_sweep(self._h, i, count, _p(self.delta) if emit else None,
                                                             self.cap, self._st))
        return self._st[0], self._st[1]

    def hub_count(self):
        nat.check("gc_shard_hub_count", self._lib.gc_shard_hub_count(self._h, self._ct.byref(self._a)))
        return self._a.value

    def start_hubs(self, i, from_slices):
        nat.check("gc_shard_start_hubs", self._lib.gc_shard_start_hubs(self._h, i, 1 if from_slices else 0,
                                                                       self._ct.byref(self._a)))
        return self._a.value

    def start_hubs_async(self, i, from_slices, grid=3):
        """the hub sweeps enqueued (``grid`` full-grid sweeps, then the one-workgroup tail);
        a checked ``finish_async`` verifies on the device that they converged"""
        nat.check("gc_shard_start_hubs_async", self._lib.gc_shard_start_hubs_async(
            self._h, i, 1 if from_slices else 0, int(grid)))
        return int(grid)

    def resume_hubs(self):
        nat.check("gc_shard_resume_hubs", self._lib.gc_shard_resume_hubs(self._h, self._ct.byref(self._a)))
        return self._a.value

    def apply_checked(self, kind, recv, r, hdr_stride):
        nat.check("gc_shard_apply_checked", self._lib.gc_shard_apply_checked(self._h, kind, _p(recv), int(recv.numel()),
                                                                             r, int(hdr_stride)))

    def clear_halt(self, code):
        nat.check("gc_shard_clear_halt", self._lib.gc_shard_clear_halt(self._h, int(code)))

    def finish_async(self, r, from_deltas=False, check=False):
        nat.check("gc_shard_finish_async", self._lib.gc_shard_finish_async(self._h, r, 1 if from_deltas else 0,
                                                                           1 if check else 0))

    def slice_buffer(self, stride):
        # one cached buffer per size (header + slice, or the bare slice of an overflow)
        if self._slice is None:
            self._slice = {}
        if stride not in self._slice:
            self._slice[stride] = torch.empty(stride, dtype=torch.uint8, device=self.device)
        return self._slice[stride]

    def get_slice(self, buf):
        nat.check("gc_shard_get_slice", self._lib.gc_shard_get_slice(self._h, _p(buf)))

    def put_slices(self, recv, stride, starts, lens):
        ct = self._ct
        a = (ct.c_int64 * len(starts))(*starts)
        b = (ct.c_int64 * len(lens))(*lens)
        nat.check("gc_shard_put_slices", self._lib.gc_shard_put_slices(self._h, _p(recv), stride, a, b, len(starts)))

    def finish(self, r, from_deltas=False):
        ct = self._ct
        nat.check("gc_shard_finish", self._lib.gc_shard_finish(self._h, r, 1 if from_deltas else 0,
                                                               ct.byref(self._a), ct.byref(self._b)))
        return self._a.value, self._b.value

    def reseed(self, r):
        ct = self._ct
        nat.check("gc_shard_reseed", self._lib.gc_shard_reseed(self._h, r, ct.byref(self._a), ct.byref(self._b)))
        return self._a.value, self._b.value

    def export_state(self, track_rounds):
        """The replicated state at a round top, in HBM (gc_shard_export): int32 tensors of the
        colours (-1 uncoloured), the rounds they were coloured in (None unless tracked) and the
        rank's OWN frontier (uncoloured vertices of [lo, hi) with a coloured listed neighbour)."""
        colors = torch.empty(max(self.n, 1), dtype=torch.int32, device=self.device)
        cround = torch.empty(max(self.n, 1), dtype=torch.int32, device=self.device) if track_rounds else None
        front = torch.empty(self.cap, dtype=torch.int32, device=self.device)
        nat.check("gc_shard_export", self._lib.gc_shard_export(self._h, _p(colors), _p(cround), _p(front),
                                                               self._ct.byref(self._a)))
        return colors[:self.n], None if cround is None else cround[:self.n], front[:self._a.value]

    def colors(self, track_rounds, fetch=True):
        """Final colours (and rounds) to host; fetch=False only settles them in HBM."""
        colors = np.empty(self.n, np.int32) if fetch else None
        cround = np.empty(self.n, np.int32) if track_rounds and fetch else None
        nat.check("gc_shard_colors", self._lib.gc_shard_colors(
            self._h, None if colors is None else colors.ctypes.data_as(self._ct.c_void_p),
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
    dense_exchanges: int = 0
    hub_halts: int = 0  # checked finishes that found the asynchronous hub JP unfinished (some rank)
    fused_misses: int = 0  # fused propose seams that could not be applied (the unfused path followed)
    ahead_misses: int = 0  # sweep seams run ahead that overflowed (the host moved their deltas)
    ahead_seams: int = 0  # sweep seams run ahead of the host
    switch_round: int = None  # hybrid_color: the round the one-GPU engine took over (None: never)

    @property
    def rounds(self):
        return len(self.round_U)

    @property
    def max_color(self):
        return int(self.colors.max()) if len(self.colors) else -1


K8_BIG = 62  # candidates >= 62 do not fit the 6-bit proposal byte (gc_internal.h)
HDR = 5      # header words carried in front of every seam's payload (GC_SEAM_HDR)
H_SWEEPS = 5  # halt code of a checked finish whose hub JP had not converged (GC_H_SWEEPS)
H_SEAM = 7    # halt code of a fused propose seam that could not be applied (GC_H_SEAM)


def _hdr_values(words):
    """int64 array [P, HDR] of header words -> their signed 32-bit values."""
    x = np.asarray(words, dtype=np.int64) & 0xFFFFFFFF
    return np.where(x >= 1 << 31, x - (1 << 32), x)


def shard_color(ops, comm, num_colors=None, e1=True, track_rounds=False, dense=None, local_sweeps=1,
                want_colors=True, inline=4096, deferred=True, hub_budget=3, fuse=True, ahead=4,
                inline_max=1 << 16, switch_below=None, round0=0, switch_after_peak=False):
    """graph_coloring (coloring.py:73) over the ranks of ``comm``; every rank returns the
    same ShardResult (records with the single-GPU semantics of gc_color).

    Each seam is ONE all-gather in the usual case: a header (the round scalars: frontier,
    max proposal, failures, undecided, count) in front of up to ``inline`` deltas, or in
    front of the rank's slice of the proposal bytes when the seam is dense.  Only when some
    rank has more deltas than fit inline does a second all-gather follow: the rest of the
    deltas, or -- when they would outweigh it (``dense=None``; True/False force it) -- every
    rank's slice, copied back in place without a scatter.  ``local_sweeps`` JP sweeps run
    between two exchanges of the sweep seam (more than one pays where neighbours are
    mostly rank-local, e.g. meshes cut into slabs).  A round whose seams all moved deltas
    ends from the received IN states (O(winners)), otherwise from a scan of the proposal
    bytes.  ``want_colors=False`` leaves the colours in HBM (``ops.colors`` fetches them).

    With an ``ops`` that has ``finish_async`` (``HipShard``), the round's end (and with
    replicated hubs their JP) is only enqueued: the winners' count comes back in word 4 of
    the next propose seam's header, so a round costs the host one wait per seam and none
    for the hubs or the commit.  A finish that found the hub JP unfinished halts on every
    rank alike (word 4 < 0): the rest of the hub sweeps run, the finish is enqueued again
    and the propose seam repeated.  ``deferred=False`` keeps the host-paced hub JP and
    finish; ``hub_budget`` is the first round's full-grid hub sweeps (then adapted).

    ``fuse``: when the last round's frontiers fit the inline deltas, the propose seam's
    all-gather, its apply and the first JP sweep seam are enqueued together, with ONE host
    wait for both headers.  The apply checks every rank's header on the device and, when
    some rank halted or overflowed, applies nothing and halts the shard (GC_H_SEAM), so the
    sweep behind it does nothing; the host clears that halt and takes the unfused path.

    ``ahead``: a fused round enqueues up to that many JP sweep seams behind the propose seam
    (as many as the last round needed), each applied on the device with the same check, and
    the host reads all their headers in its one wait.  A seam whose deltas overflowed on some
    rank halts the shard there: the host clears the halt, moves that seam's deltas itself and
    runs the sweeps behind it again.  Seams past the JP's end sweep empty lists.

    The inline part follows the frontiers: a round's is the last round's largest per-rank
    frontier rounded up to a power of two, between ``inline`` and ``inline_max`` (every rank
    derives it from the same headers), so a round whose frontier did not outgrow the last
    one's moves its deltas in one all-gather per seam and runs fused.

    ``switch_below``: stop at the top of the first round whose frontier (all ranks) is
    non-empty and smaller than that -- after the last round's finish has resolved and before
    any of this round's exchanges is applied by the host -- and return with ``switch_round``
    set (``hybrid_color`` hands the state to the one-GPU engine there).  With
    ``switch_after_peak`` only once some round's frontier reached ``switch_below`` (or after
    SWITCH_GRACE rounds): a colouring's first frontiers are the seeds' neighbours, often small,
    before the frontier peaks (R-MAT-26: the first round's is below n/64, rounds 1-3 far above).
    ``round0`` numbers the rounds of a run started from a colouring in progress."""
    k = -1 if num_colors is None else int(num_colors)
    U, _ = ops.begin(k, track_rounds)
    res = ShardResult(status=OK, colors=None, colored_round=None)
    dev = ops.delta.device
    P = comm.size
    rng = comm.gather_stats([ops.lo, ops.hi], dev)
    starts = [int(x) for x in rng[:, 0]]
    lens = [int(x) for x in rng[:, 1] - rng[:, 0]]
    stride = max(max(lens), 1)
    C0 = C = max(int(inline), 0)
    Cmax = max(int(inline_max), C0)
    # replicated hubs (gc_shard_start_hubs): the same count on every rank
    repl = getattr(ops, "hub_count", lambda: 0)() > 0
    hdr_bytes = 8 * HDR

    def rec(u, f, mm, acc, seeds):
        res.round_U.append(int(u))
        res.round_F.append(int(f))
        res.round_maxmex.append(int(mm))
        res.round_accepted.append(int(acc))
        res.round_seeds.append(int(seeds))

    def slice_for(maxc):  # a slice seam moves stride bytes per rank, deltas 8 * maxc
        return dense if dense is not None else 8 * maxc > stride

    def gather(send):
        """one all-gather of the seams' send buffers; -> (headers [P, HDR], received)."""
        res.exchanges += 1
        recv = comm.allgather(send)
        if recv.dtype == torch.int64:
            words = recv.view(P, -1)[:, :HDR]
        else:  # slice seam: header bytes in front of each rank's slice
            res.dense_exchanges += 1
            # (reshape copies unless P == 1, where the row stride need not be a multiple of 8)
            words = recv.view(P, -1)[:, :hdr_bytes].reshape(-1).view(torch.int64).view(P, HDR)
        return _hdr_values(words.cpu().numpy()), recv

    def finish_deltas(kind, hdr, recv, r, dense_ok):
        """after a delta seam: apply, or move what did not fit inline.  -> dense?"""
        maxc = int(hdr[:, 3].max())
        if maxc > C and dense_ok and slice_for(maxc):
            res.exchanges += 1
            res.dense_exchanges += 1
            buf = ops.slice_buffer(stride)
            ops.get_slice(buf)
            ops.put_slices(comm.allgather(buf), stride, starts, lens)
            return True
        ops.apply(kind, recv, int(recv.numel()), r)
        if maxc > C:
            res.exchanges += 1
            own = int(hdr[comm.rank, 3])
            rest = comm.gather_deltas(ops.delta[C:], max(own - C, 0), maxc - C)
            ops.apply(kind, rest, int(rest.numel()), r)
        return False

    max_rounds = 4 * ops.n + 16
    deferred = deferred and hasattr(ops, "finish_async")
    pending = None  # (round, U, F, maxmex, from_deltas) of a round whose finish is enqueued
    acc_known = None  # its winners, from a rank whose finish completed (when another halted)
    hub_grid, calm = max(int(hub_budget), 1), 0  # full-grid hub sweeps before the tail; rounds without a halt
    fuse_on = fuse and deferred and dense is not True and C0 > 0
    last_fmax = None  # largest per-rank frontier of the last propose seam (does the next one fit inline?)
    last_seams = 1  # sweep seams the last round needed (how many a fused round runs ahead)
    r = int(round0)
    fpeak = 0  # the largest frontier so far (switch_after_peak)
    while True:
        if U == 0 and pending is None:  # coloring.py:86-90
            rec(0, 0, -1, 0, 0)
            break
        if r > max_rounds:
            raise RuntimeError("round limit exceeded")
        if last_fmax is not None and C0 > 0:
            C = min(Cmax, max(C0, 1 << max(int(last_fmax) - 1, 0).bit_length()))
        fused = fuse_on and last_fmax is not None and last_fmax <= C
        pre = []  # sweep seams run ahead of the host: (headers, received), applied on the device
        cand_applied = False  # the propose seam's deltas were applied on the device
        if fused:
            res.exchanges += 1
            recv = comm.allgather(ops.propose_seam(r, C))
            ops.apply_checked(KIND_CAND, recv, r, HDR + C)
            recvs = [recv]
            for j in range(max(1, min(int(ahead), last_seams))):
                res.exchanges += 1
                res.ahead_seams += 1
                recvs.append(comm.allgather(ops.sweep_seam(j, 1, C, True, stride)))
                ops.apply_checked(KIND_STATE, recvs[-1], r, HDR + C)
            words = torch.stack([x.view(P, -1)[:, :HDR] for x in recvs]).cpu().numpy()  # the one host wait
            hdr = _hdr_values(words[0])
            pre = [(_hdr_values(words[j]), recvs[j]) for j in range(1, len(recvs))]
            cand_applied = int(hdr[:, 4].min()) >= 0 and int(hdr[:, 3].max()) <= C
            if not cand_applied:  # applied nowhere, and the sweep seams behind it did nothing
                ops.clear_halt(H_SEAM)  # (a rank halted by its finish keeps that halt)
                pre = []
                res.fused_misses += 1
        else:
            hdr, recv = gather(ops.propose_seam(r, C))
        if pending is not None:
            st = hdr[:, 4]
            if int(st.min()) < 0:
                # Some rank's finish found its hub JP unfinished (the ranks list their hubs in
                # different orders, so a sweep budget can suffice on one rank and not on
                # another): those ranks run the rest and finish; every rank repeats the
                # (idempotent) propose seam.  A finished rank's header holds the winners.
                assert set(int(x) for x in st[st < 0]) == {-H_SWEEPS}, f"unexpected halt codes {st}"
                if (st >= 0).any():
                    acc_known = int(st[st >= 0][0])
                if int(st[comm.rank]) < 0:
                    res.jp_sweeps += ops.resume_hubs()
                    ops.finish_async(pending[0], pending[4], check=True)
                hub_grid = min(hub_grid + 1, 8)
                calm = 0
                res.hub_halts += 1
                continue  # the propose seam again, after the finish
            acc = acc_known if acc_known is not None else int(st[0])
            acc_known = None
            calm += 1
            if calm >= 32 and hub_grid > min(2, int(hub_budget)):  # the budget has sufficed a while: trim it
                hub_grid -= 1
                calm = 0
            rec(pending[1], pending[2], pending[3], acc, 0)
            U -= acc
            pending = None
            if U == 0:
                rec(0, 0, -1, 0, 0)
                break
        F, maxmex, fails = int(hdr[:, 0].sum()), int(hdr[:, 1].max()), int(hdr[:, 2].sum())
        last_fmax = int(hdr[:, 0].max())
        fpeak = max(fpeak, F)
        if switch_below is not None and 0 < F < int(switch_below) and (
                not switch_after_peak or fpeak >= int(switch_below) or r - round0 >= SWITCH_GRACE):
            # the round's proposals and any sweeps run ahead touched no colour and no frontier
            res.switch_round = r
            break
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
        # candidates >= 62 live in cand[], outside the proposal bytes: deltas only
        if not cand_applied:
            finish_deltas(KIND_CAND, hdr, recv, r, maxmex < K8_BIG)
        # JP sweeps; a rank decides at most what it has left, so the seam's form is known
        # before the sweep runs (and a slice seam writes no deltas)
        i, left, any_dense, hubs_async, seams = 0, int(hdr[:, 0].max()), False, False, 0
        while True:
            if pre:  # a sweep seam run ahead (fused with the propose seam)
                sl, cnt = False, 1
                hdr, recv = pre.pop(0)
                if int(hdr[:, 3].max()) > C:
                    # some rank's deltas overflowed: applied nowhere, the shard halted there and
                    # the seams behind it did nothing (their sweeps run again from i + 1)
                    ops.clear_halt(H_SEAM)
                    pre = []
                    res.ahead_misses += 1
                    any_dense |= finish_deltas(KIND_STATE, hdr, recv, r, True)
                i += 1
            else:
                sl = slice_for(left)
                cnt = local_sweeps if i else 1
                hdr, recv = gather(ops.sweep_seam(i, cnt, C, not sl, stride))
                i += cnt
                if sl:
                    ops.put_slices(recv[hdr_bytes:], hdr_bytes + stride, starts, lens)
                    any_dense = True
                else:
                    any_dense |= finish_deltas(KIND_STATE, hdr, recv, r, True)
            seams += 1
            if int(hdr[:, 0].sum()) == 0:
                break
            if repl and int(hdr[:, 2].sum()) == 0:
                # every rank's lights are decided: each rank runs the hubs' sweeps alike
                i += len(pre)  # (sweeps run ahead past the lights' end swept empty lists)
                if deferred:
                    res.jp_sweeps += ops.start_hubs_async(i, any_dense, hub_grid)
                    hubs_async = True
                else:
                    res.jp_sweeps += ops.start_hubs(i, any_dense)
                break
            left = int(hdr[:, 0].max())
            res.jp_sweeps += 1
        last_seams = seams
        if deferred:
            ops.finish_async(r, not any_dense, check=hubs_async)
            pending = (r, U, F, maxmex, not any_dense)
        else:
            acc, _ = ops.finish(r, not any_dense)
            rec(U, F, maxmex, acc, 0)
            U -= acc
        r += 1
    res.colors, res.colored_round = ops.colors(track_rounds, want_colors)
    return res


def engine_resume(dg, lock=None):
    """``resume`` for ``hybrid_color``: the one-GPU engine (DeviceGraph.resume, gc_color_resume)
    continues from the replicated state; ``lock`` serialises ranks that share ``dg`` (threads)."""
    def run(colors, cround, front, round0, num_colors, e1, track_rounds, want_colors):
        # the state (and the all-gathered frontier) are produced on torch's stream: the engine's
        # first read waits on that stream (an event), not on the host
        stream = torch.cuda.current_stream(colors.device).cuda_stream if colors.is_cuda else None
        args = (colors.data_ptr(), front.data_ptr() if front.numel() else None, int(front.numel()), int(round0))
        kw = dict(cround_dev=cround.data_ptr() if (track_rounds and cround is not None) else None,
                  num_colors=num_colors, e1=e1, want_rounds=True, want_colors=want_colors, stream=stream)
        if lock is None:
            return dg.resume(*args, **kw)
        with lock:
            return dg.resume(*args, **kw)
    return run


def hybrid_color(ops, comm, resume, switch_below, num_colors=None, e1=True, track_rounds=False, want_colors=True,
                 **kw):
    """graph_coloring (coloring.py:73) over the ranks while the frontier is large, then on
    every rank's own GPU alone: ``shard_color`` runs the sharded rounds until a round's
    frontier (all ranks) drops below ``switch_below``; there every rank exports the
    replicated colours and its own part of the frontier, the parts are all-gathered (the
    ranges are disjoint: their union is the frontier) and ``resume`` -- the one-GPU engine
    (``engine_resume``) -- runs the remaining rounds from that state on each rank alike.  The
    long tail of small rounds then costs no exchange at all, while the big rounds are split
    over the ranks.  Every rank returns the same ShardResult: the sharded rounds' records
    followed by the engine's, the colours bit-identical to one GPU (LFMIS under the global
    rank does not depend on where a round runs)."""
    res = shard_color(ops, comm, num_colors, e1, track_rounds, want_colors=False, switch_below=switch_below, **kw)
    if res.switch_round is None:  # finished (or failed / stalled) before the frontier got small
        res.colors, res.colored_round = ops.colors(track_rounds, want_colors)
        return res
    colors, cround, front = ops.export_state(track_rounds)
    counts = [int(x) for x in comm.gather_stats([front.numel()], colors.device)[:, 0]]
    m = max(max(counts), 1)
    send = torch.full((m,), -1, dtype=torch.int32, device=front.device)
    send[:front.numel()].copy_(front)
    allf = comm.allgather(send).view(comm.size, m)
    front = torch.cat([allf[p, :counts[p]] for p in range(comm.size)])
    tail = resume(colors, cround, front, res.switch_round, num_colors, e1, track_rounds, want_colors)
    for key in ("U", "F", "maxmex", "accepted", "seeds"):
        getattr(res, "round_" + key).extend(int(x) for x in getattr(tail, "round_" + key))
    res.status, res.fail_round, res.fail_count = int(tail.status), int(tail.fail_round), int(tail.fail_count)
    res.reseeds += int(tail.reseeds)
    res.jp_sweeps += int(tail.jp_sweeps)
    res.colors = tail.colors
    res.colored_round = tail.colored_round if track_rounds else None
    return res


def color_threads(dg, parts, num_colors=None, e1=True, track_rounds=False, switch_below=None, **kw):
    """``parts`` shards of one colouring on the current GPU, driven by threads: the test
    and rehearsal path of the multi-GPU engine on one device."""
    rp, _ = dg.export()
    ranges = balanced_ranges(rp, parts)
    hub = ThreadHub(parts)
    # the CSR is read-only: every shard borrows it, each keeps its own replicated state
    shards = [HipShard(dg, lo, hi) for lo, hi in ranges]
    out = [None] * parts
    err = []

    lock = threading.Lock()

    def run(i):
        try:
            comm = ThreadTransport(hub, i)
            if switch_below is None:
                out[i] = shard_color(shards[i], comm, num_colors, e1, track_rounds, **kw)
            else:
                out[i] = hybrid_color(shards[i], comm, engine_resume(dg, lock), switch_below, num_colors, e1,
                                      track_rounds, **kw)
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
