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
