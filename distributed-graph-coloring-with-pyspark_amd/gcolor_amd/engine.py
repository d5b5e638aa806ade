"""Device-resident graphs and the colouring / validation entry points (C-ABI wrappers).

``DeviceGraph`` replaces the reference's persisted RDD of ``Node`` objects
(coloring.py:201-209) with an HBM-resident CSR; ``DeviceGraph.color`` replaces
``graph_coloring(graph_rdd, numOfColors, sc)`` (coloring.py:73, variant B
coloring_optimized.py:70) and ``DeviceGraph.validate`` replaces
``validate_graph_coloring`` (coloring.py:149-162).  All compute runs in libgcolor.so.
"""
import contextlib
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as nat

ROUND_CAP = 1 << 17


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def is_symmetric(rp, col):
    """True iff (v,u) listed <=> (u,v) listed (as sets); host-side, small graphs."""
    n = len(rp) - 1
    if n == 0:
        return True
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    dst = col.astype(np.int64)
    a = np.unique(src * n + dst)
    b = np.unique(dst * n + src)
    return a.shape == b.shape and bool(np.array_equal(a, b))


@dataclass
class ColorResult:
    status: int
    colors: np.ndarray
    colored_round: np.ndarray
    rounds: int
    round_U: np.ndarray
    round_F: np.ndarray
    round_maxmex: np.ndarray
    round_accepted: np.ndarray
    round_seeds: np.ndarray
    fail_round: int
    fail_count: int
    reseeds: int
    max_color: int
    jp_sweeps: int
    device_ms: float
    kernels: dict = field(default_factory=dict)
    async_aborts: int = 0  # asynchronous JP launches that handed their rest to host sweeps (0 expected)
    hubs: int = 0  # vertices with pushed hub state (0: no hub, or the hub index did not fit)
    core_rounds: int = 0  # rounds whose hub JP the hub core decided in one workgroup (csrc/gc_core.hip)

    @property
    def ok(self):
        return self.status == nat.GC_OK

    @property
    def num_colors(self):
        return self.max_color + 1

    @property
    def balg_bytes(self):
        """SURVEY.md §8d algorithmic bytes of the colouring (validate pass excluded)."""
        return sum(k["bytes"] for k in self.kernels.values())


@contextlib.contextmanager
def _input_stream(lib, stream):
    """gc_set_input_stream around one call (per thread; restored to the device-wide wait)."""
    if stream is None:
        yield
        return
    nat.check("gc_set_input_stream", lib.gc_set_input_stream(ctypes.c_void_p(int(stream)), 1))
    try:
        yield
    finally:
        lib.gc_set_input_stream(None, 0)


class DeviceGraph:
    """An HBM-resident CSR graph (file positions; adjacency exactly as listed)."""

    def __init__(self, handle):
        self._lib = nat.load()
        self._h = handle
        n, nnz, md = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        fl = ctypes.c_uint32()
        nat.check("gc_graph_info", self._lib.gc_graph_info(self._h, ctypes.byref(n), ctypes.byref(nnz),
                                                            ctypes.byref(md), ctypes.byref(fl)))
        self.n, self.nnz, self.max_degree, self.flags = n.value, nnz.value, md.value, fl.value
        dev = ctypes.c_int32()
        nat.check("gc_graph_device", self._lib.gc_graph_device(self._h, ctypes.byref(dev)))
        self.device_index = dev.value  # the HIP device the graph lives on

    # ---- construction -------------------------------------------------------------------
    @classmethod
    def from_csr(cls, rp, col, symmetric=None):
        lib = nat.load()
        rp = np.ascontiguousarray(rp, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        n = rp.shape[0] - 1
        if symmetric is None:
            symmetric = is_symmetric(rp, col) if col.shape[0] <= 20_000_000 else False
        h = ctypes.c_void_p()
        nat.check("gc_graph_create", lib.gc_graph_create(_ptr(rp), _ptr(col), n, col.shape[0],
                                                         nat.GC_GRAPH_SYMMETRIC if symmetric else 0,
                                                         ctypes.byref(h)))
        return cls(h)

    @classmethod
    def from_device(cls, d_row_ptr, d_col, n, nnz, symmetric=False, stream=None):
        """A graph from a CSR already resident in HBM: device pointers (ints, e.g. a torch
        tensor's ``data_ptr()``) to int64[n+1] offsets and int32[nnz] positions.  The rows are
        read in place and rank-partitioned into the graph's own array (gc_graph_create_device).
        ``stream``: the hipStream_t (int, e.g. ``torch.cuda.current_stream().cuda_stream``) the
        CSR was written on -- the first read waits for that stream only; None waits for the
        whole device."""
        lib = nat.load()
        h = ctypes.c_void_p()
        with _input_stream(lib, stream):
            nat.check("gc_graph_create_device", lib.gc_graph_create_device(
                ctypes.c_void_p(d_row_ptr), ctypes.c_void_p(d_col), int(n), int(nnz),
                nat.GC_GRAPH_SYMMETRIC if symmetric else 0, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def rmat(cls, scale, edge_factor=16, a=0.57, b=0.19, c=0.19, seed=1):
        lib = nat.load()
        h = ctypes.c_void_p()
        nat.check("gc_graph_create_rmat", lib.gc_graph_create_rmat(scale, edge_factor, a, b, c, seed, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def mesh(cls, nx, ny, nz):
        lib = nat.load()
        h = ctypes.c_void_p()
        nat.check("gc_graph_create_mesh", lib.gc_graph_create_mesh(nx, ny, nz, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def uniform(cls, n, max_degree, seed=42):
        rp, col = uniform_csr(n, max_degree, seed)
        return cls.from_csr(rp, col, symmetric=True)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gc_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def symmetric(self):
        return bool(self.flags & nat.GC_GRAPH_SYMMETRIC)

    def export(self, col=True):
        """Host copy of the device CSR (rows as the engine stores them); col=False copies
        only the row offsets (returns (rp, None))."""
        rp = np.empty(self.n + 1, np.int64)
        c = np.empty(max(self.nnz, 1), np.int32) if col else None
        nat.check("gc_graph_export", self._lib.gc_graph_export(self._h, _ptr(rp), _ptr(c)))
        return rp, (c[: self.nnz] if col else None)

    def export_device(self, d_row_ptr, d_col):
        """Device-to-device copy of the CSR (rows as the engine stores them) into caller-owned
        device buffers (pointers as ints; either may be None)."""
        nat.check("gc_graph_export_device", self._lib.gc_graph_export_device(
            self._h, ctypes.c_void_p(d_row_ptr) if d_row_ptr else None, ctypes.c_void_p(d_col) if d_col else None))

    def lower_counts(self):
        """nlow[v]: entries at the head of exported row v that rank below v (deg, pos)."""
        out = np.empty(max(self.n, 1), np.int32)
        nat.check("gc_graph_lower_counts", self._lib.gc_graph_lower_counts(self._h, _ptr(out)))
        return out[: self.n]

    # ---- hot path -------------------------------------------------------------------------
    def color(self, variant="A", num_colors=None, e1=True, kernel_timing=False, want_rounds=True,
              want_colors=True, priority=None, speculative=False):
        """graph_coloring(graph, numOfColors): returns ColorResult.  ``num_colors=None``
        is unbounded; on a bounded failure ``colors`` is the round-start snapshot.
        ``priority=None`` keeps the reference's (deg, pos) tie-break (coloring.py:64); an
        int seed ranks each colour's conflict resolution by the seeded priority
        prio_hash(seed, v) instead (variant A).  ``speculative=True``: speculative
        first-fit rounds with one-shot resolution under that rank (variant A)."""
        opt = nat.GcOptions(variant=nat.GC_VARIANT_A if variant == "A" else nat.GC_VARIANT_B,
                            e1=1 if e1 else 0, num_colors=-1 if num_colors is None else int(num_colors),
                            kernel_timing=_timing_mask(kernel_timing),
                            priority=nat.GC_PRIORITY_REF if priority is None else nat.GC_PRIORITY_SEEDED,
                            seed=0 if priority is None else int(priority) & (2**64 - 1),
                            speculative=1 if speculative else 0, reserved=0)
        return self._color(opt, want_rounds, want_colors, ROUND_CAP)

    def resume(self, colors_dev, front_dev, nfront, round0, cround_dev=None, num_colors=None, e1=True,
               want_rounds=True, want_colors=True, kernel_timing=False, stream=None):
        """The colouring continued from round ``round0`` of a run in progress (gc_color_resume):
        the rest of graph_coloring's loop (coloring.py:85-132) from a round start.
        ``colors_dev`` / ``cround_dev`` / ``front_dev`` are DEVICE pointers (ints) of int32 arrays
        -- the colours so far (-1 uncoloured), the round each was coloured in (or None), and the
        ``nfront`` uncoloured vertices with a coloured listed neighbour.  Variant A, reference
        rank.  The records are those of rounds round0, round0 + 1, ...  ``stream``: as in
        from_device, the stream those buffers were written on (None: the whole device)."""
        opt = nat.GcOptions(variant=nat.GC_VARIANT_A, e1=1 if e1 else 0,
                            num_colors=-1 if num_colors is None else int(num_colors),
                            kernel_timing=_timing_mask(kernel_timing), priority=nat.GC_PRIORITY_REF, seed=0,
                            speculative=0, reserved=0)
        args = (ctypes.c_void_p(colors_dev), ctypes.c_void_p(cround_dev) if cround_dev else None,
                ctypes.c_void_p(front_dev) if front_dev else None, int(nfront), int(round0))
        with _input_stream(self._lib, stream):
            return self._color(opt, want_rounds, want_colors, ROUND_CAP, resume=args)

    def _color(self, opt, want_rounds, want_colors, cap, resume=None):
        st = nat.GcStats()
        cap = cap if want_rounds else 0
        rb = {k: np.zeros(max(cap, 1), np.int64) for k in ("U", "F", "maxmex", "accepted", "seeds")}
        if want_rounds:
            st.round_cap = cap
            for k, arr in rb.items():
                setattr(st, "round_" + k, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        colors = np.empty(self.n, np.int32) if want_colors else None
        cround = np.empty(self.n, np.int32) if want_colors else None
        if resume is None:
            status = self._lib.gc_color(self._h, ctypes.byref(opt), _ptr(colors), _ptr(cround), ctypes.byref(st))
        else:
            status = self._lib.gc_color_resume(self._h, ctypes.byref(opt), *resume, _ptr(colors), _ptr(cround),
                                               ctypes.byref(st))
        nat.check("gc_color_resume" if resume else "gc_color", status, ok=(nat.GC_OK, nat.GC_FAILED, nat.GC_STALLED))
        r = st.rounds
        if want_rounds and r > cap:  # more rounds than the buffers hold (long paths): once more, sized
            return self._color(opt, want_rounds, want_colors, int(r), resume=resume)
        kernels = {}
        for i, name in enumerate(nat.KERNEL_CLASSES):
            kernels[name] = {"launches": int(st.k_launches[i]), "ms": float(st.k_ms[i]), "bytes": float(st.k_bytes[i])}
        return ColorResult(status=status, colors=colors, colored_round=cround, rounds=r,
                           round_U=rb["U"][:r].copy() if want_rounds else None,
                           round_F=rb["F"][:r].copy() if want_rounds else None,
                           round_maxmex=rb["maxmex"][:r].copy() if want_rounds else None,
                           round_accepted=rb["accepted"][:r].copy() if want_rounds else None,
                           round_seeds=rb["seeds"][:r].copy() if want_rounds else None,
                           fail_round=st.fail_round, fail_count=st.fail_count, reseeds=st.reseeds,
                           max_color=st.max_color, jp_sweeps=st.jp_sweeps, device_ms=st.device_ms,
                           kernels=kernels, async_aborts=int(st.async_aborts), hubs=int(st.hubs),
                           core_rounds=int(st.core_rounds))

    def validate(self, colors=None, lo=None, hi=None):
        """validate_graph_coloring counts on the device (coloring.py:149-162): (#uncoloured,
        #conflicting listed pairs).
        ``colors=None`` validates the last colouring still resident on the device.  ``lo`` /
        ``hi``: the counts of the rows of vertices [lo, hi) only (gc_validate_range; disjoint
        ranges covering the graph add up to the whole graph's counts)."""
        u, c = ctypes.c_int64(), ctypes.c_int64()
        arr = None if colors is None else np.ascontiguousarray(colors, dtype=np.int32)
        if lo is None and hi is None:
            nat.check("gc_validate", self._lib.gc_validate(self._h, _ptr(arr), ctypes.byref(u), ctypes.byref(c)))
        else:
            lo = 0 if lo is None else int(lo)
            hi = self.n if hi is None else int(hi)
            nat.check("gc_validate_range", self._lib.gc_validate_range(self._h, _ptr(arr), lo, hi, ctypes.byref(u),
                                                                       ctypes.byref(c)))
        return u.value, c.value


def release_cache():
    """Give the library's parked device blocks back to the runtime (gc_release_cache).  The
    allocator keeps freed blocks for the next graph of the same size (up to 64 GB by default;
    GC_ALLOC_IDLE_CAP_GB / GC_ALLOC_IDLE_RESERVE_GB raise it, csrc/gc_alloc.hip); call this
    before handing a large share of HBM to another allocator (torch)."""
    nat.check("gc_release_cache", nat.load().gc_release_cache())


def _timing_mask(kernel_timing):
    """True = every kernel class; a class name or list of names = only those."""
    if not kernel_timing:
        return 0
    if kernel_timing is True:
        return 0xFF
    names = [kernel_timing] if isinstance(kernel_timing, str) else list(kernel_timing)
    return sum(1 << nat.KERNEL_CLASSES.index(k) for k in names)


def uniform_csr(n, max_degree, seed=42):
    """Native graph.py:30-43 process (splitmix64 stream) on the host, as CSR."""
    lib = nat.load()
    rp = np.empty(n + 1, np.int64)
    col = np.empty(max(n * max_degree, 1), np.int32)
    nnz = ctypes.c_int64()
    nat.check("gc_gen_uniform", lib.gc_gen_uniform(n, max_degree, seed, _ptr(rp), _ptr(col), col.shape[0],
                                                   ctypes.byref(nnz)))
    return rp, col[: nnz.value].copy()


def device_count():
    lib = nat.load()
    c = ctypes.c_int32()
    nat.check("gc_device_count", lib.gc_device_count(ctypes.byref(c)))
    return c.value
