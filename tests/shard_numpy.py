"""CPU stand-in for gcolor_amd.shard.HipShard (TEST INFRASTRUCTURE ONLY).

Same phase interface and delta format as the HIP shard, computed with numpy/Python on
the rank's replicated copy of the state, so the multi-rank driver
(gcolor_amd.shard.shard_color) and its torch.distributed / thread transports can be
tested on CPU (gloo).  The phase semantics restate coloring.py:44-70, 114-127 (see
oracle/gcolor_oracle.c): the frontier is recomputed from the colours (uncoloured with a
coloured listed neighbour), independently of the GPU's push-based frontier.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import _components_argmax  # noqa: E402

UND, IN, OUT = 0, 1, 2


class NumpyShard:
    def __init__(self, rp, col, lo, hi):
        self.rp = np.asarray(rp, np.int64)
        self.col = np.asarray(col, np.int64)
        self.n = len(self.rp) - 1
        self.lo, self.hi = int(lo), int(hi)
        self.deg = np.diff(self.rp)
        self.adj = [self.col[self.rp[v]:self.rp[v + 1]].tolist() for v in range(self.n)]
        key = [(int(self.deg[v]), v) for v in range(self.n)]
        self.lower = [[u for u in self.adj[v] if key[u] < key[v]] for v in range(self.n)]
        self.delta = torch.empty(max(self.hi - self.lo, 1), dtype=torch.int64)

    # delta entries: vertex << 32 | value (value as unsigned 32 bits)
    def _emit(self, pairs):
        for i, (v, val) in enumerate(pairs):
            self.delta[i] = (v << 32) | (val & 0xFFFFFFFF)
        return len(pairs)

    @staticmethod
    def _decode(recv, tot):
        if recv is None or not tot:
            return []
        out = []
        for e in recv[:tot].tolist():
            v = e >> 32
            if v < 0:
                continue
            val = e & 0xFFFFFFFF
            out.append((v, val - (1 << 32) if val >= 1 << 31 else val))
        return out

    def _owned(self, v):
        return self.lo <= v < self.hi

    def _frontier(self):
        c = self.c
        return [v for v in range(self.lo, self.hi) if c[v] == -1 and any(c[u] >= 0 for u in self.adj[v])]

    def begin(self, k, track):
        self.k, self.track = k, track
        self.c = np.where(self.deg == 0, 0, -1).astype(np.int64)
        self.cround = np.where(self.deg == 0, 0, -1).astype(np.int64)
        seed = None
        for v in range(self.n):                       # coloring.py:21-22, ties -> last
            if self.c[v] == -1 and (seed is None or self.deg[v] >= self.deg[seed]):
                seed = v
        if seed is not None:
            self.c[seed], self.cround[seed] = 0, 0
        self.cand = np.full(self.n, -1, np.int64)
        self.state = np.zeros(self.n, np.int64)
        return int((self.c == -1).sum()), len(self._frontier())

    def propose(self, r):
        self.cand[:] = -1
        self.state[:] = UND
        self.F = self._frontier()
        pairs, mm, fails = [], -1, 0
        for v in self.F:
            used = {int(self.c[u]) for u in self.adj[v] if self.c[u] >= 0}
            mex = 0
            while mex in used:
                mex += 1
            self.cand[v] = mex
            mm = max(mm, mex)
            if self.k >= 0 and mex >= self.k:
                fails += 1
            pairs.append((v, mex))
        return self._emit(pairs), len(self.F), mm, fails

    # ---- seams (gcolor_amd.shard.HipShard's interface): header words + inline deltas ----
    @staticmethod
    def _words(vals):
        return [((0xFFFFFFFF << 32) | (int(x) & 0xFFFFFFFF)) - (1 << 64) for x in vals]

    def _pack(self, vals, cnt, C):
        H = len(vals)
        send = torch.full((H + C,), -1, dtype=torch.int64)
        send[:H] = torch.tensor(self._words(vals), dtype=torch.int64)
        k = min(cnt, C)
        if k:
            send[H:H + k] = self.delta[:k]
        return send

    def propose_seam(self, r, C):
        cnt, f, mm, fails = self.propose(r)
        return self._pack([f, mm, fails, cnt, 0], cnt, C)

    def sweep_seam(self, i, count, C, emit, stride):
        cnt, und = self.sweep(i, count, emit)
        if emit:
            return self._pack([und, cnt, 0, cnt, 0], cnt, C)
        buf = torch.zeros(40 + stride, dtype=torch.uint8)
        buf[:40] = torch.tensor(self._words([und, 0, 0, 0, 0]), dtype=torch.int64).view(torch.uint8)
        self.get_slice(buf[40:])
        return buf

    def apply(self, kind, recv, tot, r):
        for v, val in self._decode(recv, tot):
            if self._owned(v):
                continue
            if kind == 0:
                self.cand[v], self.state[v] = val, UND
            elif kind == 1:
                self.state[v] = val
            else:
                self._colour(v, val, r)

    def _colour(self, v, val, r):
        self.c[v] = val
        self.cand[v] = -1
        if self.track:
            self.cround[v] = r + 1

    def sweep(self, i, count=1, emit=True):
        pairs = []
        for j in range(i, i + count):
            todo = self.F if j == 0 else self.und
            und = []
            for v in todo:
                f = 0
                for u in self.lower[v]:
                    if self.cand[u] == self.cand[v] and self.cand[u] >= 0:
                        f |= 1 if self.state[u] == IN else (2 if self.state[u] == UND else 0)
                if f & 1:
                    self.state[v] = OUT
                    pairs.append((v, OUT))
                elif f & 2:
                    und.append(v)
                else:
                    self.state[v] = IN
                    pairs.append((v, IN))
            self.und = und
        return (self._emit(pairs) if emit else 0), len(self.und)

    # dense seam: proposal bytes cand6 << 2 | state (63 = no candidate), the rank's slice
    def slice_buffer(self, stride):
        return torch.zeros(stride, dtype=torch.uint8)

    def get_slice(self, buf):
        c = self.cand[self.lo:self.hi]
        c6 = np.where(c < 0, 63, np.minimum(c, 62))  # 62: the candidate is in cand (BIG)
        buf[:self.hi - self.lo] = torch.from_numpy(((c6 << 2) | self.state[self.lo:self.hi]).astype(np.uint8))

    def put_slices(self, recv, stride, starts, lens):
        for p, (s0, ln) in enumerate(zip(starts, lens)):
            if ln <= 0 or (s0 == self.lo and ln == self.hi - self.lo):  # own slice
                continue
            b = recv[p * stride:p * stride + ln].numpy().astype(np.int64)
            c6 = b >> 2
            cur = self.cand[s0:s0 + ln]
            self.cand[s0:s0 + ln] = np.where(c6 == 63, -1, np.where(c6 == 62, cur, c6))
            self.state[s0:s0 + ln] = b & 3

    def finish(self, r, from_deltas=False):
        # every proposer's final state is replicated: all ranks colour all winners
        win = [v for v in range(self.n) if self.state[v] == IN and self.cand[v] >= 0]
        for v in win:
            self._colour(v, int(self.cand[v]), r)
        return len(win), len(self._frontier())

    def reseed(self, r):
        seeds = _components_argmax(self.adj, self.deg.tolist(), self.c.tolist())
        for s in seeds:
            self.c[s] = 0
            self.cround[s] = r + 1
        return len(seeds), len(self._frontier())

    def colors(self, track, fetch=True):
        if not fetch:
            return None, None
        return self.c.astype(np.int32), (self.cround.astype(np.int32) if track else None)

    def export_state(self, track):
        """HipShard.export_state: the replicated colours (and rounds) and the OWN frontier."""
        return (torch.from_numpy(self.c.astype(np.int32)),
                torch.from_numpy(self.cround.astype(np.int32)) if track else None,
                torch.tensor(self._frontier(), dtype=torch.int32))


class DeferredNumpyShard(NumpyShard):
    """The stand-in with HipShard's enqueue-only round end and fused propose seam
    (gcolor_amd.shard.shard_color with finish_async): the round's winners travel in word 4
    of the next propose seam's header, and a fused seam's apply checks every rank's header
    first -- when one cannot be applied (a rank's deltas overflowed the inline part) the
    shard 'halts' (GC_H_SEAM): the sweep behind it does nothing until the host clears it."""

    HDR = 5

    def begin(self, k, track):
        self.acc_last, self.halted = 0, False
        return super().begin(k, track)

    def finish_async(self, r, from_deltas=False, check=False):
        self.acc_last, _ = self.finish(r, from_deltas)

    def propose_seam(self, r, C):
        cnt, f, mm, fails = self.propose(r)
        return self._pack([f, mm, fails, cnt, self.acc_last], cnt, C)

    def apply_checked(self, kind, recv, r, hdr_stride):
        if self.halted:
            return
        words = recv.view(-1, hdr_stride)[:, :self.HDR].numpy() & 0xFFFFFFFF
        vals = np.where(words >= 1 << 31, words - (1 << 32), words)
        if (vals[:, 4] < 0).any() or (vals[:, 3] > hdr_stride - self.HDR).any():
            self.halted = True
            return
        self.apply(kind, recv, int(recv.numel()), r)

    def clear_halt(self, code):
        self.halted = False

    def sweep_seam(self, i, count, C, emit, stride):
        if self.halted:  # the sweep does nothing; its header is ignored by the host
            return self._pack([0, 0, 0, 0, 0], 0, C)
        return super().sweep_seam(i, count, C, emit, stride)


class InflatedShard(DeferredNumpyShard):
    """DeferredNumpyShard whose sweep seams carry every delta three times (applying a state
    twice changes nothing): their counts can overflow the inline part while the propose
    seam's fit, which exercises the host's recovery of a sweep seam run ahead."""

    def __init__(self, rp, col, lo, hi):
        super().__init__(rp, col, lo, hi)
        self.delta = torch.empty(3 * max(self.hi - self.lo, 1), dtype=torch.int64)
        self._x3 = False

    def _emit(self, pairs):
        return super()._emit(pairs * 3 if self._x3 else pairs)

    def sweep(self, i, count=1, emit=True):
        self._x3 = True
        try:
            return super().sweep(i, count, emit)
        finally:
            self._x3 = False


class ResumedNumpyShard(DeferredNumpyShard):
    """One rank over every vertex, started from a colouring in progress: the stand-in for the
    one-GPU engine's gc_color_resume in gcolor_amd.shard.hybrid_color."""

    def __init__(self, rp, col, colors, cround):
        super().__init__(rp, col, 0, len(rp) - 1)
        self._c0 = np.asarray(colors, np.int64).copy()
        self._r0 = None if cround is None else np.asarray(cround, np.int64).copy()

    def begin(self, k, track):
        self.acc_last, self.halted = 0, False
        self.k, self.track = k, track
        self.c = self._c0.copy()
        self.cround = self._r0.copy() if self._r0 is not None else np.where(self.c >= 0, 0, -1)
        self.cand = np.full(self.n, -1, np.int64)
        self.state = np.zeros(self.n, np.int64)
        return int((self.c == -1).sum()), len(self._frontier())


def numpy_resume(rp, col, calls=None):
    """``resume`` for hybrid_color on CPU: checks that the all-gathered frontier is exactly the
    frontier of the exported colours, then runs the remaining rounds on one stand-in rank."""
    from gcolor_amd import shard as shm

    def run(colors, cround, front, round0, num_colors, e1, track_rounds, want_colors):
        ops = ResumedNumpyShard(rp, col, colors.numpy(), None if cround is None else cround.numpy())
        ops.c = ops._c0
        got = front.tolist()
        assert len(got) == len(set(got)) and sorted(got) == ops._frontier(), "exported frontier"
        if calls is not None:
            calls.append((int(round0), len(got)))
        return shm.shard_color(ops, shm.ThreadTransport(shm.ThreadHub(1), 0), num_colors, e1, track_rounds,
                               round0=round0)
    return run
