"""Colouring states that drive k_commit into its corner cases -- TEST INFRASTRUCTURE.

stage_overflow_case: a round whose winners are packed into the first wave chunks of the
frontier, each winner with many unclaimed neighbours, so the waves holding them overflow their
LDS stage (GC_STAGE_CAP entries) and flush mid-launch while the workgroups with no chunk have
already taken their arrival tickets on the same counter (the ticket-closing commit:
gc_stage_flush_ticket).  Round 3's fault on the 10M uniform graph with the asynchronous JP (a
memory aperture violation in k_commit) is this case: the mid-launch flush took its base from the
ticketed count, 2^40 per finished workgroup.
"""
import numpy as np


def stage_overflow_case(K, leaves, n):
    """Centres 0..K-1, centre i with anchor K + i (pre-coloured 0) and `leaves` private leaves;
    every other vertex isolated (coloured 0).  Returns (rp, col, colors, front, expected): the
    frontier is the K centres in order; the colouring ends two rounds later with every centre
    colour 1 (its candidate mex{0}) and every leaf colour 0 (mex{1}): `expected` holds the
    final colours and the two rounds' records (F, accepted)."""
    assert n >= 2 * K + K * leaves
    c = np.arange(K, dtype=np.int64)
    lv = 2 * K + np.arange(K * leaves, dtype=np.int64)
    owner = np.repeat(c, leaves)
    src = np.concatenate([c, K + c, np.repeat(c, leaves), lv])
    dst = np.concatenate([K + c, c, lv, owner])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    rp = np.cumsum(rp)
    col = dst.astype(np.int32)
    colors = np.zeros(n, np.int32)
    colors[:K] = -1
    colors[2 * K:2 * K + K * leaves] = -1
    front = c.astype(np.int32)
    final = np.zeros(n, np.int32)
    final[:K] = 1
    expected = {"colors": final, "F": [K, K * leaves], "accepted": [K, K * leaves],
                "U": [K + K * leaves, K * leaves]}
    return rp, col, colors, front, expected


def _csr(n, src, dst):
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, src + 1, 1)
    return np.cumsum(rp), dst.astype(np.int32)


def stage_overflow_tree(fanout, levels, n):
    """The same corner from a plain colouring (no resume): a rooted tree -- the root with
    fanout + 2 children, every other inner vertex with fanout children (degree fanout + 1, so
    the root is the unique seed) -- padded with isolated vertices to n.  Round k's frontier is
    level k + 1: every vertex wins (siblings are never adjacent) and claims its children, so a
    wave holding a chunk of one level pushes chunk x fanout entries.  Vertex ids: the root 0,
    then the levels in order.  Returns (rp, col, expected) with expected colours (level parity:
    even levels and the isolated vertices 0, odd levels 1) and the per-round frontiers."""
    sizes = [1, fanout + 2]
    while len(sizes) < levels:
        sizes.append(sizes[-1] * fanout)
    starts = np.cumsum([0] + sizes)
    assert starts[-1] <= n
    src, dst = [], []
    for lv in range(1, levels):
        child = np.arange(starts[lv], starts[lv + 1], dtype=np.int64)
        k = fanout + 2 if lv == 1 else fanout
        parent = starts[lv - 1] + (child - starts[lv]) // k
        src += [parent, child]
        dst += [child, parent]
    rp, col = _csr(n, np.concatenate(src), np.concatenate(dst))
    colors = np.zeros(n, np.int32)
    for lv in range(levels):
        colors[starts[lv]:starts[lv + 1]] = lv & 1
    return rp, col, {"colors": colors, "F": sizes[1:], "levels": sizes}
