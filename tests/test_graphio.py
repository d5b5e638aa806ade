"""Graph files, host only -- no GPU.

* The native JSON reader (gc_json_read_graph) against graph.py:15-28's own rules,
  restated in graphio.load_graph_json_py: same (ids, CSR) on what it accepts, and on
  every other input the same exception type and text as the Python path -- which is
  what coloring.py:179-181 prints after "Error loading graph: ".
* The json.dump(indent=4) writers byte-identical to Python's encoder.
* The binary CSR (.gcsr) round trip and its header / range checks.
"""
import json
import random

import numpy as np
import pytest

from conftest import golden_names, load_golden

from gcolor_amd import _native, graphio


def outcome(fn, path):
    try:
        ids, rp, col = fn(path)
        return ("ok", [int(i) if not isinstance(i, (float, bool, str)) and i is not None else i for i in ids],
                rp.tolist(), col.tolist())
    except Exception as e:  # noqa: BLE001 -- the CLI catches Exception too (coloring.py:179)
        return ("err", type(e).__name__, str(e))


def same_as_python(path):
    a = outcome(graphio.load_graph_json, path)
    b = outcome(graphio.load_graph_json_py, path)
    assert a == b
    return a


def native_status(path):
    lib = _native.load()
    import ctypes
    ptr = ctypes.POINTER(_native.GcCsr)()
    st = lib.gc_json_read_graph(str(path).encode(), ctypes.byref(ptr))
    if st == 0:
        lib.gc_csr_free(ptr)
    return st


@pytest.mark.parametrize("name", [n for n in golden_names()])
def test_native_reader_matches_python_on_golden_graphs(name, tmp_path):
    rec = load_golden(name)
    p = tmp_path / "g.json"
    p.write_text(json.dumps([{"id": i, "neighbors": nb, "color": -1} for i, nb in rec["graph"]], indent=4))
    res = same_as_python(p)
    if res[0] == "ok":
        assert native_status(p) == 0  # integer ids: taken natively, not through the fallback


def _random_graph_text(rng, n, ids, indent):
    nodes = []
    for i in range(n):
        nb = [ids[rng.randrange(n)] for _ in range(rng.randrange(6))] if n else []
        d = {"id": ids[i], "neighbors": nb, "color": rng.choice([-1, 3, 0])}
        if rng.random() < 0.3:  # key order and extra keys do not matter (graph.py reads two keys)
            d = {"color": d["color"], "extra": {"a": [1, 2.5e3, None, True, "x\\u00e9\\n"]}, "neighbors": nb,
                 "id": ids[i]}
        nodes.append(d)
    return json.dumps(nodes, indent=indent)


@pytest.mark.parametrize("seed", range(12))
def test_native_reader_random_ids_and_layouts(seed, tmp_path):
    rng = random.Random(seed)
    n = rng.choice([0, 1, 5, 50, 300])
    pool = [rng.randrange(-2**63, 2**63) for _ in range(n)]
    if seed % 3 == 0:
        pool = list(range(n))  # identity ids (the fast path)
    if seed % 4 == 1 and n > 2:
        pool[1] = pool[0]  # repeated id: the LAST node carrying it wins (graph.py:23)
    text = _random_graph_text(rng, n, pool, rng.choice([None, 0, 2, 4, "\t"]))
    p = tmp_path / "g.json"
    p.write_text(text)
    res = same_as_python(p)
    assert res[0] == "ok"
    assert native_status(p) == 0


CASES = {
    "string_ids": '[{"id": "a", "neighbors": ["b"]}, {"id": "b", "neighbors": []}]',
    "float_id_matches_int": '[{"id": 1.0, "neighbors": [1]}]',
    "bool_id": '[{"id": true, "neighbors": [1]}]',
    "huge_int": '[{"id": 123456789012345678901234567890, "neighbors": []}]',
    "missing_neighbor": '[{"id": 0, "neighbors": [0, 7]}, {"id": 1, "neighbors": [5]}]',
    "missing_neighbor_negative": '[{"id": 0, "neighbors": [-3]}]',
    "missing_id_key": '[{"neighbors": []}]',
    "missing_neighbors_key": '[{"id": 0}]',
    "top_level_dict": '{"id": 0, "neighbors": []}',
    "top_level_int": '5',
    "element_not_object": '[[0, 1]]',
    "neighbors_string": '[{"id": 0, "neighbors": "0"}]',
    "neighbors_null": '[{"id": 0, "neighbors": null}]',
    "duplicate_key": '[{"id": 0, "id": 1, "neighbors": [1]}]',
    "escaped_key": '[{"\\u0069d": 0, "neighbors": []}]',
    "trailing_comma": '[{"id": 0, "neighbors": [],}]',
    "truncated": '[{"id": 0, "neighbors": [',
    "extra_data": '[] []',
    "empty_list": '[]',
    "empty_file": '',
    "nan_color": '[{"id": 0, "neighbors": [], "color": NaN}]',
    "leading_zero": '[{"id": 01, "neighbors": []}]',
    "minus_zero": '[{"id": -0, "neighbors": [0]}]',
    "bom": '﻿[]',
    "unicode_value": '[{"id": 0, "neighbors": [], "name": "é"}]',
    "control_char_in_string": '[{"id": 0, "neighbors": [], "s": "a\tb"}]',
    "unhashable_id": '[{"id": [1], "neighbors": []}]',
    "self_loop_and_dups": '[{"id": 4, "neighbors": [4, 4, 9]}, {"id": 9, "neighbors": []}]',
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_native_reader_edge_cases_match_python(name, tmp_path):
    p = tmp_path / "g.json"
    p.write_bytes(CASES[name].encode("utf-8"))
    res = same_as_python(p)
    if name == "missing_neighbor":
        assert res == ("err", "KeyError", "7")
    if name in ("self_loop_and_dups", "minus_zero", "empty_list"):
        assert res[0] == "ok" and native_status(p) == 0


def test_missing_file_message_matches_python(tmp_path):
    p = tmp_path / "nope.json"
    assert outcome(graphio.load_graph_json, p) == outcome(graphio.load_graph_json_py, p)
    assert outcome(graphio.load_graph, p) == outcome(graphio.load_graph_json_py, p)


@pytest.mark.parametrize("seed", range(6))
def test_writers_byte_identical_to_json_dump(seed, tmp_path):
    rng = random.Random(seed)
    n = rng.choice([0, 1, 7, 200])
    ids = [rng.randrange(-2**63, 2**63) if seed % 2 else i for i in range(n)]
    adj = [[rng.randrange(n) for _ in range(rng.randrange(5))] for _ in range(n)]
    rp, col = graphio.csr_from_adjacency(adj)
    colors = [rng.randrange(-3, 40) for _ in range(n)]
    a, b = tmp_path / "a.json", tmp_path / "b.json"
    graphio.write_coloring_json(str(a), ids, colors)
    with open(b, "w") as f:
        json.dump([{"id": v, "color": c} for v, c in zip(ids, colors)], f, indent=4)
    assert a.read_bytes() == b.read_bytes()
    graphio.write_graph_json(str(a), np.asarray(ids, np.int64), rp, col)
    with open(b, "w") as f:
        json.dump([{"id": ids[i], "neighbors": [ids[u] for u in adj[i]], "color": -1} for i in range(n)], f, indent=4)
    assert a.read_bytes() == b.read_bytes()
    graphio.write_graph_json(str(a), ids, rp, col, colors=colors)
    with open(b, "w") as f:
        json.dump([{"id": ids[i], "neighbors": [ids[u] for u in adj[i]], "color": colors[i]} for i in range(n)], f,
                  indent=4)
    assert a.read_bytes() == b.read_bytes()


def test_writer_keeps_python_path_for_non_int_ids(tmp_path):
    ids = ["a", 2.5, True]
    a = tmp_path / "a.json"
    graphio.write_coloring_json(str(a), ids, [0, 1, 2])
    assert json.loads(a.read_text()) == [{"id": "a", "color": 0}, {"id": 2.5, "color": 1}, {"id": True, "color": 2}]


@pytest.mark.parametrize("with_ids", [False, True])
@pytest.mark.parametrize("n", [0, 1, 1000])
def test_gcsr_roundtrip(tmp_path, n, with_ids):
    rng = np.random.default_rng(n)
    deg = rng.integers(0, 9, n)
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(deg)
    col = rng.integers(0, max(n, 1), int(rp[-1])).astype(np.int32)
    ids = rng.integers(-2**62, 2**62, n) if with_ids else None
    p = tmp_path / "g.gcsr"
    graphio.write_csr(str(p), rp, col, ids=ids, symmetric=True)
    assert graphio.is_gcsr(str(p))
    ids2, rp2, col2, flags = graphio.read_csr(str(p))
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and flags == _native.GC_GRAPH_SYMMETRIC
    assert (ids2 is None) if not with_ids else np.array_equal(ids, ids2)
    ids3, rp3, _ = graphio.load_graph(str(p))
    assert np.array_equal(rp3, rp) and len(ids3) == n


def test_gcsr_rejects_corrupt_files(tmp_path):
    rp = np.array([0, 2, 3], np.int64)
    col = np.array([1, 1, 0], np.int32)
    p = tmp_path / "g.gcsr"
    graphio.write_csr(str(p), rp, col)
    good = p.read_bytes()
    bad_col = bytearray(good)
    bad_col[32 + 24:32 + 28] = (5).to_bytes(4, "little")  # col[0] = 5 >= n
    for blob in (good[:-4], bytes(bad_col), b"GCSR\0\0\0\2" + good[8:]):
        q = tmp_path / "bad.gcsr"
        q.write_bytes(blob)
        with pytest.raises(_native.GcolorError):
            graphio.read_csr(str(q))


def test_json_to_gcsr_to_json_bytes(tmp_path):
    """JSON -> .gcsr (with ids) -> JSON reproduces the reference's serialised bytes."""
    random.seed(3)
    from gcolor_amd.generators import reference_graph
    adj = reference_graph(300, 6)
    rp, col = graphio.csr_from_adjacency(adj)
    ids = [10 * i - 77 for i in range(300)]
    a = tmp_path / "a.json"
    graphio.write_graph_json(str(a), ids, rp, col)
    ids1, rp1, col1 = graphio.load_graph(str(a))
    g = tmp_path / "a.gcsr"
    graphio.write_csr(str(g), rp1, col1, ids=ids1)
    ids2, rp2, col2 = graphio.load_graph(str(g))
    b = tmp_path / "b.json"
    graphio.write_graph_json(str(b), ids2, rp2, col2)
    assert a.read_bytes() == b.read_bytes()
