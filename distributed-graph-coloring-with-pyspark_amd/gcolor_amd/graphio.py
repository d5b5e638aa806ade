"""Graph / colouring files with the reference's exact schema and error behaviour.

* ``load_graph_json`` follows graph.py:15-28: nodes in file order, neighbour ids
  resolved through a dict built from every node (a repeated id resolves to the LAST
  node carrying it), a missing id raises ``KeyError`` (the CLI prints
  "Error loading graph: <e>" and exits 1, coloring.py:177-181); the input ``color`` is
  ignored (graph.py:20).  The native reader (``gc_json_read_graph``, csrc/gc_io_host.cpp)
  parses the common case -- integer ids -- in one pass over an mmap of the file; files it
  does not take (string / float / boolean ids, malformed JSON, ...) are re-read here with
  Python's ``json`` and graph.py's own linking, which raise the reference's exceptions.
* ``write_coloring_json`` writes ``[{"id", "color"}]`` with ``json.dump(indent=4)``
  (coloring.py:238-241) -- byte-identical to the reference for the same colours.
* ``write_graph_json`` writes ``[{"id", "neighbors", "color"}]`` with indent=4
  (graph.py:10-12 via node.py:8-13).
* ``read_csr`` / ``write_csr``: the binary CSR file (``.gcsr``, layout in
  csrc/gc_io_host.cpp) for graphs past JSON scale; ``load_graph`` picks the format from
  the file's magic bytes.
"""
import ctypes
import json

import numpy as np

GCSR_MAGIC = b"GCSR\x00\x00\x00\x01"
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def csr_from_adjacency(adj):
    """adjacency as lists of positions -> (rp int64[n+1], col int32[nnz])."""
    rp = np.zeros(len(adj) + 1, np.int64)
    if adj:
        rp[1:] = np.cumsum(np.fromiter((len(a) for a in adj), dtype=np.int64, count=len(adj)))
    col = np.fromiter((u for a in adj for u in a), dtype=np.int32, count=int(rp[-1]))
    return rp, col


def _lib():
    from . import _native
    return _native, _native.load()


def _take_csr(native, lib, ptr):
    """Copy a library-owned gc_csr into numpy arrays and free it."""
    c = ptr.contents
    try:
        n, nnz = int(c.n), int(c.nnz)
        rp = np.ctypeslib.as_array(c.row_ptr, shape=(n + 1,)).copy()
        col = np.ctypeslib.as_array(c.col, shape=(max(nnz, 1),))[:nnz].copy()
        ids = np.ctypeslib.as_array(c.ids, shape=(max(n, 1),))[:n].copy() if c.ids else None
        return ids, rp, col, int(c.flags)
    finally:
        lib.gc_csr_free(ptr)


def load_graph_json_py(path):
    """graph.py:15-28 restated over positions (Python json; any id type)."""
    with open(path, "r") as f:
        node_data = json.load(f)
    ids = [data["id"] for data in node_data]
    pos = {vid: i for i, vid in enumerate(ids)}
    adj = [[pos[nid] for nid in data["neighbors"]] for data in node_data]
    rp, col = csr_from_adjacency(adj)
    return ids, rp, col


def load_graph_json(path, native=True):
    """Returns (ids, rp, col).  Raises exactly what graph.py:15-28 raises."""
    if native:
        nat, lib = _lib()
        ptr = ctypes.POINTER(nat.GcCsr)()
        st = lib.gc_json_read_graph(str(path).encode(), ctypes.byref(ptr))
        if st == nat.GC_OK:
            ids, rp, col, _ = _take_csr(nat, lib, ptr)
            return ids, rp, col
        if st == nat.GC_EKEY:  # graph.py:25: node_dict[neighbor_id]
            raise KeyError(int(lib.gc_last_error().decode()))
        if st != nat.GC_EUNSUPPORTED:
            if st == nat.GC_EIO:  # open() failed: let Python raise its own OSError text
                open(path, "r").close()
            nat.check("gc_json_read_graph", st)
    return load_graph_json_py(path)


def read_csr(path):
    """.gcsr -> (ids or None, rp, col, flags)."""
    nat, lib = _lib()
    ptr = ctypes.POINTER(nat.GcCsr)()
    nat.check("gc_csr_read", lib.gc_csr_read(str(path).encode(), ctypes.byref(ptr)))
    return _take_csr(nat, lib, ptr)


def write_csr(path, rp, col, ids=None, symmetric=False):
    nat, lib = _lib()
    rp = np.ascontiguousarray(rp, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    n = len(rp) - 1
    idp = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, np.int64)
        assert len(ids) == n
        idp = ids.ctypes.data
    nat.check("gc_csr_write", lib.gc_csr_write(str(path).encode(), rp.ctypes.data, col.ctypes.data, idp, n,
                                               len(col), nat.GC_GRAPH_SYMMETRIC if symmetric else 0))


def is_gcsr(path):
    with open(path, "rb") as f:
        return f.read(8) == GCSR_MAGIC


def load_graph(path):
    """(ids, rp, col) from a reference JSON graph or a .gcsr file (by magic bytes)."""
    ids, rp, col, _ = load_graph_ex(path)
    return ids, rp, col


def load_graph_ex(path):
    """(ids, rp, col, symmetric): symmetric is the .gcsr writer's assertion (True/False),
    or None for JSON (the engine then checks the lists itself)."""
    if is_gcsr(path):
        ids, rp, col, flags = read_csr(path)
        ids = np.arange(len(rp) - 1, dtype=np.int64) if ids is None else ids
        from . import _native
        return ids, rp, col, bool(flags & _native.GC_GRAPH_SYMMETRIC)
    ids, rp, col = load_graph_json(path)
    return ids, rp, col, None


def _int64_ids(ids):
    """ids as an int64 array when every id is a plain int in range, else None."""
    if isinstance(ids, np.ndarray) and ids.dtype.kind in "iu":
        return np.ascontiguousarray(ids, np.int64)
    if all(type(v) is int and _I64_MIN <= v <= _I64_MAX for v in ids):
        return np.asarray(ids, np.int64) if len(ids) else np.zeros(0, np.int64)
    return None


def write_coloring_json(path, ids, colors):
    ids64 = _int64_ids(ids)
    if ids64 is not None:
        nat, lib = _lib()
        c = np.ascontiguousarray(colors, np.int32)
        nat.check("gc_json_write_coloring",
                  lib.gc_json_write_coloring(str(path).encode(), ids64.ctypes.data, c.ctypes.data, len(ids64)))
        return
    result = [{"id": vid, "color": int(c)} for vid, c in zip(ids, colors)]
    with open(path, "w") as f:
        json.dump(result, f, indent=4)


def write_graph_json(path, ids, rp, col, colors=None):
    ids64 = _int64_ids(ids)
    if ids64 is not None:
        nat, lib = _lib()
        rp = np.ascontiguousarray(rp, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        c = np.ascontiguousarray(colors, np.int32) if colors is not None else None
        nat.check("gc_json_write_graph", lib.gc_json_write_graph(str(path).encode(), ids64.ctypes.data,
                                                                 rp.ctypes.data, col.ctypes.data, len(ids64),
                                                                 c.ctypes.data if c is not None else None))
        return
    out = []
    for i, vid in enumerate(ids):
        nb = [ids[u] for u in col[rp[i]:rp[i + 1]]]
        out.append({"id": vid, "neighbors": nb, "color": -1 if colors is None else int(colors[i])})
    with open(path, "w") as f:
        json.dump(out, f, indent=4)
