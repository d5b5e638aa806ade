"""ctypes binding of libgcolor.so (the C-ABI declared in include/gcolor.h).

The library is built in-tree (``make -C distributed-graph-coloring-with-pyspark_amd/csrc``
or ``__graft_entry__.build()``) and loaded from ``gcolor_amd/lib/libgcolor.so``.  There is
no fallback: if the library is missing or no GPU is present the calls fail loudly.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "lib", "libgcolor.so")
# measurement builds of the same sources with other compile-time settings
# (tools/build_variant.sh); never a fallback: the path must exist
if os.environ.get("GC_LIB_PATH"):
    LIB_PATH = os.environ["GC_LIB_PATH"]
CSRC = os.path.join(PKG_DIR, "csrc")

GC_OK, GC_FAILED, GC_STALLED = 0, 1, 2
GC_EINVAL, GC_EHIP, GC_ENOMEM, GC_ERCCL, GC_EROUNDS = -1, -2, -3, -4, -5
GC_EUNSUPPORTED, GC_EKEY, GC_EIO = -6, -7, -8
GC_GRAPH_SYMMETRIC = 1
GC_VARIANT_A, GC_VARIANT_B = 0, 1
GC_NKERNELS = 8
KERNEL_CLASSES = ["init", "propose", "resolve", "sweep", "commit", "reseed", "validate", "other"]

# Every symbol include/gcolor.h declares (checked by tests/test_abi.py).
EXPORTS = ["gc_graph_create", "gc_graph_create_device", "gc_graph_create_rmat", "gc_graph_create_mesh",
           "gc_graph_destroy", "gc_graph_info", "gc_graph_device", "gc_graph_export", "gc_graph_export_device", "gc_graph_lower_counts", "gc_color", "gc_color_resume", "gc_validate", "gc_validate_range",
           "gc_gen_uniform", "gc_last_error", "gc_release_cache", "gc_set_input_stream", "gc_device_count", "gc_set_device",
           "gc_shard_create", "gc_shard_destroy", "gc_shard_begin", "gc_shard_propose", "gc_shard_apply",
           "gc_shard_sweep", "gc_shard_finish", "gc_shard_reseed", "gc_shard_colors", "gc_shard_set_stream",
           "gc_shard_propose_async", "gc_shard_sweep_async", "gc_shard_pack",
           "gc_shard_get_slice", "gc_shard_put_slices", "gc_shard_hub_count", "gc_shard_start_hubs",
           "gc_shard_start_hubs_async", "gc_shard_resume_hubs", "gc_shard_finish_async",
           "gc_shard_apply_checked", "gc_shard_clear_halt", "gc_shard_export",
           "gc_json_read_graph", "gc_json_write_coloring", "gc_json_write_graph", "gc_csr_write", "gc_csr_read",
           "gc_csr_free"]


GC_PRIORITY_REF, GC_PRIORITY_SEEDED = 0, 1


class GcOptions(ctypes.Structure):
    _fields_ = [("variant", ctypes.c_int32), ("e1", ctypes.c_int32), ("num_colors", ctypes.c_int64),
                ("kernel_timing", ctypes.c_int32), ("priority", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("speculative", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_I64P = ctypes.POINTER(ctypes.c_int64)


class GcCsr(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("row_ptr", ctypes.POINTER(ctypes.c_int64)),
                ("col", ctypes.POINTER(ctypes.c_int32)), ("ids", ctypes.POINTER(ctypes.c_int64)),
                ("flags", ctypes.c_uint32)]


class GcStats(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_int64), ("fail_round", ctypes.c_int64), ("fail_count", ctypes.c_int64),
                ("reseeds", ctypes.c_int64), ("max_color", ctypes.c_int64), ("jp_sweeps", ctypes.c_int64),
                ("device_ms", ctypes.c_double),
                ("k_launches", ctypes.c_int64 * GC_NKERNELS), ("k_ms", ctypes.c_double * GC_NKERNELS),
                ("k_bytes", ctypes.c_double * GC_NKERNELS),
                ("round_cap", ctypes.c_int64), ("round_U", _I64P), ("round_F", _I64P),
                ("round_maxmex", _I64P), ("round_accepted", _I64P), ("round_seeds", _I64P),
                ("async_aborts", ctypes.c_int64), ("hubs", ctypes.c_int64), ("core_rounds", ctypes.c_int64)]


class GcolorError(RuntimeError):
    def __init__(self, fn, status, msg):
        super().__init__(f"{fn} failed (status {status}): {msg}")
        self.status = status


_lib = None


def build(jobs=8):
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"], check=True)


def load():
    """Load libgcolor.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P, I32, I64, U32, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "gc_graph_create": ([P, P, I64, I64, U32, PP], ctypes.c_int),
        "gc_graph_create_device": ([P, P, I64, I64, U32, PP], ctypes.c_int),
        "gc_graph_create_rmat": ([I32, I32, ctypes.c_double, ctypes.c_double, ctypes.c_double, U64, PP], ctypes.c_int),
        "gc_graph_create_mesh": ([I64, I64, I64, PP], ctypes.c_int),
        "gc_graph_destroy": ([P], None),
        "gc_graph_info": ([P, _I64P, _I64P, _I64P, ctypes.POINTER(U32)], ctypes.c_int),
        "gc_graph_device": ([P, ctypes.POINTER(I32)], ctypes.c_int),
        "gc_graph_export": ([P, P, P], ctypes.c_int),
        "gc_graph_export_device": ([P, P, P], ctypes.c_int),
        "gc_graph_lower_counts": ([P, P], ctypes.c_int),
        "gc_color": ([P, ctypes.POINTER(GcOptions), P, P, ctypes.POINTER(GcStats)], ctypes.c_int),
        "gc_color_resume": ([P, ctypes.POINTER(GcOptions), P, P, P, I64, I64, P, P, ctypes.POINTER(GcStats)],
                            ctypes.c_int),
        "gc_validate": ([P, P, _I64P, _I64P], ctypes.c_int),
        "gc_validate_range": ([P, P, I64, I64, _I64P, _I64P], ctypes.c_int),
        "gc_gen_uniform": ([I64, I32, U64, P, P, I64, _I64P], ctypes.c_int),
        "gc_last_error": ([], ctypes.c_char_p),
        "gc_release_cache": ([], ctypes.c_int),
        "gc_set_input_stream": ([P, ctypes.c_int32], ctypes.c_int),
        "gc_device_count": ([ctypes.POINTER(I32)], ctypes.c_int),
        "gc_set_device": ([I32], ctypes.c_int),
        "gc_shard_create": ([P, I64, I64, PP], ctypes.c_int),
        "gc_shard_destroy": ([P], None),
        "gc_shard_begin": ([P, I64, I32, _I64P, _I64P], ctypes.c_int),
        "gc_shard_propose": ([P, I64, P, I64, _I64P], ctypes.c_int),
        "gc_shard_apply": ([P, I32, P, I64, I64], ctypes.c_int),
        "gc_shard_sweep": ([P, I32, I32, P, I64, _I64P], ctypes.c_int),
        "gc_shard_get_slice": ([P, P], ctypes.c_int),
        "gc_shard_put_slices": ([P, P, I64, _I64P, _I64P, I32], ctypes.c_int),
        "gc_shard_finish": ([P, I64, I32, _I64P, _I64P], ctypes.c_int),
        "gc_shard_set_stream": ([P, P], ctypes.c_int),
        "gc_shard_propose_async": ([P, I64, P, I64], ctypes.c_int),
        "gc_shard_sweep_async": ([P, I32, I32, P, I64], ctypes.c_int),
        "gc_shard_pack": ([P, I32, I32, P, P, I64], ctypes.c_int),
        "gc_shard_reseed": ([P, I64, _I64P, _I64P], ctypes.c_int),
        "gc_shard_colors": ([P, P, P], ctypes.c_int),
        "gc_shard_export": ([P, P, P, P, _I64P], ctypes.c_int),
        "gc_shard_hub_count": ([P, _I64P], ctypes.c_int),
        "gc_shard_start_hubs": ([P, I32, I32, _I64P], ctypes.c_int),
        "gc_shard_start_hubs_async": ([P, I32, I32, I32], ctypes.c_int),
        "gc_shard_resume_hubs": ([P, _I64P], ctypes.c_int),
        "gc_shard_finish_async": ([P, I64, I32, I32], ctypes.c_int),
        "gc_shard_apply_checked": ([P, I32, P, I64, I64, I64], ctypes.c_int),
        "gc_shard_clear_halt": ([P, I32], ctypes.c_int),
        "gc_json_read_graph": ([ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(GcCsr))], ctypes.c_int),
        "gc_json_write_coloring": ([ctypes.c_char_p, P, P, I64], ctypes.c_int),
        "gc_json_write_graph": ([ctypes.c_char_p, P, P, P, I64, P], ctypes.c_int),
        "gc_csr_write": ([ctypes.c_char_p, P, P, P, I64, I64, U32], ctypes.c_int),
        "gc_csr_read": ([ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(GcCsr))], ctypes.c_int),
        "gc_csr_free": ([ctypes.POINTER(GcCsr)], None),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(fn_name, status, ok=(GC_OK,)):
    if status in ok:
        return status
    msg = _lib.gc_last_error().decode(errors="replace") if _lib is not None else ""
    raise GcolorError(fn_name, status, msg)
