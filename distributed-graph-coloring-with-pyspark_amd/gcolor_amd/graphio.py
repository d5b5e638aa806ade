"""JSON graph / colouring I/O with the reference's exact schema and error behaviour.

* ``load_graph_json`` follows graph.py:15-28: nodes in file order, neighbour ids
  resolved through a dict built from every node (a repeated id resolves to the LAST
  node carrying it), a missing id raises ``KeyError`` (the CLI prints
  "Error loading graph: <e>" and exits 1, coloring.py:177-181); the input ``color`` is
  ignored (graph.py:20).
* ``write_coloring_json`` writes ``[{"id", "color"}]`` with ``json.dump(indent=4)``
  (coloring.py:238-241) -- byte-identical to the reference for the same colours.
* ``write_graph_json`` writes ``[{"id", "neighbors", "color"}]`` with indent=4
  (graph.py:10-12 via node.py:8-13).
"""
import json

import numpy as np


def csr_from_adjacency(adj):
    """adjacency as lists of positions -> (rp int64[n+1], col int32[nnz])."""
    rp = np.zeros(len(adj) + 1, np.int64)
    if adj:
        rp[1:] = np.cumsum(np.fromiter((len(a) for a in adj), dtype=np.int64, count=len(adj)))
    col = np.fromiter((u for a in adj for u in a), dtype=np.int32, count=int(rp[-1]))
    return rp, col


def load_graph_json(path):
    """Returns (ids, rp, col).  Raises exactly what graph.py:15-28 raises."""
    with open(path, "r") as f:
        node_data = json.load(f)
    ids = [data["id"] for data in node_data]
    pos = {vid: i for i, vid in enumerate(ids)}
    adj = [[pos[nid] for nid in data["neighbors"]] for data in node_data]
    rp, col = csr_from_adjacency(adj)
    return ids, rp, col


def write_coloring_json(path, ids, colors):
    result = [{"id": vid, "color": int(c)} for vid, c in zip(ids, colors)]
    with open(path, "w") as f:
        json.dump(result, f, indent=4)


def write_graph_json(path, ids, rp, col, colors=None):
    out = []
    for i, vid in enumerate(ids):
        nb = [ids[u] for u in col[rp[i]:rp[i + 1]]]
        out.append({"id": vid, "neighbors": nb, "color": -1 if colors is None else int(colors[i])})
    with open(path, "w") as f:
        json.dump(out, f, indent=4)
