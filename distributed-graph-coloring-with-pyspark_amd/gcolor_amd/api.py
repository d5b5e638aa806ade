"""In-process mirror of the reference's hot-path functions.

``graph_coloring(graph, numOfColors, sc=None)``  <- coloring.py:73 (variant B:
coloring_optimized.py:70).  ``graph`` is what the reference's RDD holds -- an iterable
of ``Node`` objects in partition order -- or a ``DeviceGraph``.  Returns
``(bool, graph)`` like the reference: on failure the colours are the snapshot at the
start of the failing round.  Node colours are written back in place, as
``color_node`` does (coloring.py:37-41).

``validate_graph_coloring(graph) -> bool``  <- coloring.py:149-162, same prints.

Both run on the GPU through libgcolor.so; ``sc`` (the SparkContext) is accepted and
ignored.
"""
from .engine import DeviceGraph
from .graphio import csr_from_adjacency


def _nodes_to_device(nodes):
    pos = {}
    for i, nd in enumerate(nodes):
        pos[nd.id] = i
    adj = [[pos[nb.id] for nb in nd.neighbors] for nd in nodes]
    rp, col = csr_from_adjacency(adj)
    return DeviceGraph.from_csr(rp, col)


def graph_coloring(graph, numOfColors, sc=None, variant="A"):
    k = None if numOfColors is None else int(numOfColors)
    if isinstance(graph, DeviceGraph):
        res = graph.color(variant, num_colors=k)
        return res.status == 0, res
    nodes = list(graph)
    with _nodes_to_device(nodes) as dg:
        res = dg.color(variant, num_colors=k)
    for nd, c in zip(nodes, res.colors):
        nd.color = int(c)
    return res.status == 0, nodes


def validate_graph_coloring(graph, colors=None):
    if isinstance(graph, DeviceGraph):
        unc, conf = graph.validate(colors)
    else:
        nodes = list(graph)
        cols = [nd.color for nd in nodes]
        with _nodes_to_device(nodes) as dg:
            unc, conf = dg.validate(cols)
    if unc > 0:
        print(f"Graph coloring failed: {unc} nodes have no colors.")
        return False
    if conf > 0:
        print(f"Graph coloring failed: {conf} conflicts detected.")
        return False
    return True
