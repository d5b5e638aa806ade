"""Model of the asynchronous Jones-Plassmann round (csrc/gc_kernels.hip k_sweep_async's light
passes) -- TEST INFRASTRUCTURE.

A round's resolution (coloring.py:56-70) is the LFMIS of the proposers under the rank
(deg asc, pos asc): v keeps its candidate iff no LISTED neighbour of lower rank that kept the
same candidate exists.  k_sweep_async evaluates it with no barrier: every wave owns a static
slice of the undecided vertices and passes over its pending ones, each from its cursor (the
first lower-rank same-candidate neighbour it found undecided), until none is left, reading
the other waves' states as they happen to be.  A state only moves UND -> IN / OUT, so a
stale read only ever shows UND.  This model runs those rules vertex by vertex under a seeded
random interleaving of waves, with every read of another vertex's state taken, at random,
from an older snapshot, and colours whole graphs round by round (init, seed, E1 re-seeds as
oracle/gcolor_oracle.c).  tests/test_jp_model.py checks it equals the oracle's variant A bit
for bit: "staleness delays a decision, never changes it", the argument DESIGN §5 makes for
the asynchronous JP -- with hubs (the engine's case) and without (the lights-only rules).
"""
import random

UND, IN, OUT = 0, 1, 2


def _mex(s):
    m = 0
    while m in s:
        m += 1
    return m


def _seed(n, deg, colour):
    """oracle seed_vertex: the uncoloured vertex of largest degree, ties -> later."""
    best = None
    for v in range(n):
        if colour[v] == -1 and (best is None or deg[v] >= deg[best]):
            best = v
    return best


def _e1(n, adj, deg, colour):
    """oracle e1_reseed: per component of the uncoloured-induced subgraph (listed edges,
    either direction), its argmax (deg, pos) vertex gets colour 0.  Returns the seeds."""
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for v in range(n):
        if colour[v] != -1:
            continue
        for u in adj[v]:
            if colour[u] != -1:
                continue
            a, b = find(v), find(u)
            if a != b:
                parent[max(a, b)] = min(a, b)
    best = {}
    for v in range(n):
        if colour[v] == -1:
            r = find(v)
            if r not in best or deg[v] >= deg[best[r]]:
                best[r] = v
    return sorted(best.values())


def jp_round(adj, rank, cand, props, rng, waves=5, stale=0.3, snap_every=3, hubs=frozenset()):
    """One round's resolution over the proposers `props` as the asynchronous waves evaluate
    it; returns the set that keeps its candidate.  With `hubs` (the hub JP, gc_hubs.hip):
    the lights resolve first -- no light ever looks at a hub, every hub ranks above every
    light -- and each light winner raises the kill flag of every hub that lists it and
    proposes its colour; once every light has decided, a killed hub is OUT and the others
    resolve among themselves the same way (their lower-rank listed hubs, stale reads)."""
    st = {v: UND for v in props}
    # the lower-rank listed neighbours proposing the same candidate, in row order (the
    # engine's rows list them first; a cursor resumes at the first one found undecided)
    low = {v: [u for u in adj[v] if u in st and u != v and rank[u] < rank[v] and cand[u] == cand[v]] for v in props}
    cur = {v: 0 for v in props}
    snaps = [dict(st)]

    def read(x):
        return rng.choice(snaps)[x] if rng.random() < stale else st[x]

    def settle(order):
        nonlocal snaps
        slices = [order[i * len(order) // waves:(i + 1) * len(order) // waves] for i in range(waves)]
        pending = [list(sl) for sl in slices]
        steps = 0
        while any(pending):
            w = rng.choice([i for i in range(waves) if pending[i]])
            v = pending[w].pop(0)
            row, out, first = low[v], False, None
            for i in range(cur[v], len(row)):
                s = read(row[i])
                if s == IN:
                    out = True
                    break
                if s == UND and first is None:
                    first = i
            if out:
                st[v] = OUT
            elif first is not None:
                cur[v] = first
                pending[w].append(v)
            else:
                st[v] = IN
            steps += 1
            if steps % snap_every == 0:
                snaps.append(dict(st))
                if len(snaps) > 6:
                    snaps.pop(1)
            if steps > 200 * (len(props) + 1) ** 2:
                raise RuntimeError("the JP model does not converge")

    lights = [v for v in props if v not in hubs]
    hub_props = [v for v in props if v in hubs]
    settle(lights)
    if hub_props:
        # every light has decided (the hubs wait for the lights' counter): kill flags
        killed = {x for x in hub_props if any(u in st and u not in hubs and st[u] == IN and cand[u] == cand[x]
                                              for u in adj[x])}
        for x in killed:
            st[x] = OUT
        # a hub's scan covers its lower-rank listed hubs only (hlow); lights are the flags' part
        for x in hub_props:
            low[x] = [u for u in low[x] if u in hubs]
        snaps = [dict(st)]
        settle([x for x in hub_props if x not in killed])
    return {v for v in props if st[v] == IN}


def model_color_a(rp, col, seed=0, waves=5, stale=0.3, hub_t=None):
    """Variant A (coloring.py), unbounded, E1 on, every round's resolution by jp_round
    (hubs: deg > hub_t, None = no hub JP).  Returns (colours, per-round (U, F, accepted,
    seeds))."""
    rng = random.Random(seed)
    n = len(rp) - 1
    adj = [[int(u) for u in col[rp[v]:rp[v + 1]]] for v in range(n)]
    deg = [len(a) for a in adj]
    rank = {v: (deg[v], v) for v in range(n)}
    colour = [0 if deg[v] == 0 else -1 for v in range(n)]
    s = _seed(n, deg, colour)
    if s is not None:
        colour[s] = 0
    recs = []
    while True:
        unc = [v for v in range(n) if colour[v] == -1]
        if not unc:
            recs.append((0, 0, 0, 0))
            return colour, recs
        cand, props = {}, []
        for v in unc:
            cs = {colour[u] for u in adj[v] if colour[u] >= 0}
            if cs:
                cand[v] = _mex(cs)
                props.append(v)
        if not props:  # E1 re-seed round
            seeds = _e1(n, adj, deg, colour)
            for x in seeds:
                colour[x] = 0
            recs.append((len(unc), 0, 0, len(seeds)))
            continue
        hubs = frozenset(v for v in props if hub_t is not None and deg[v] > hub_t)
        keep = jp_round(adj, rank, cand, props, rng, waves, stale, hubs=hubs)
        for v in keep:
            colour[v] = cand[v]
        recs.append((len(unc), len(props), len(keep), 0))
        if len(recs) > 4 * n + 16:
            raise RuntimeError("round limit")
