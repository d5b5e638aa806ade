"""Graph generators.

``reference_graph`` replays graph.py:30-43 call for call on Python's ``random`` module
(``randint(0, D)`` per node, ``choice`` over the node sequence per draw), so after
``random.seed(s)`` it yields the reference's graph bit for bit.  The only change is a
guard for SURVEY Q5 (the reference spins forever when no admissible partner exists):
after many consecutive rejections it checks whether any admissible partner is left and
stops growing the node if none is; the check draws no random numbers, so every graph
the reference can finish is reproduced unchanged.

Large synthetic inputs (BASELINE configs C2-C5) come from the native generators:
``engine.uniform_csr`` (same process, splitmix64 stream, host C++),
``DeviceGraph.rmat`` and ``DeviceGraph.mesh`` (on the GPU).
"""
import random as _random

from .graphio import csr_from_adjacency


def reference_graph(node_count, max_degree, rng=_random):
    """Adjacency lists (ids == positions 0..n-1) of Graph(node_count, max_degree)."""
    n, D = node_count, max_degree
    nbrs = [[] for _ in range(n)]
    member = [set() for _ in range(n)]
    seq = range(n)
    guard = 64 * (D + 1) + 4096
    for v in range(n):
        degree = rng.randint(0, D)
        rejects = 0
        while len(nbrs[v]) < degree:
            u = rng.choice(seq)
            if u != v and u not in member[v] and len(nbrs[u]) < D:
                nbrs[v].append(u)
                member[v].add(u)
                nbrs[u].append(v)
                member[u].add(v)
                rejects = 0
                continue
            rejects += 1
            if rejects > guard:
                if not any(w != v and w not in member[v] and len(nbrs[w]) < D for w in range(n)):
                    break
                rejects = 0
    return nbrs


def reference_csr(node_count, max_degree, rng=_random):
    return csr_from_adjacency(reference_graph(node_count, max_degree, rng))
