"""Model of variant B's asynchronous fold (csrc/gc_variant_b.hip k_b_async) -- TEST INFRASTRUCTURE.

The GPU's fold (coloring_optimized.py:120-126, 168-200) is the fixpoint of two monotone
evaluations per candidate class: adm(v) (UND -> IN admitted at arrival / OUT refused) and, for
admitted u, ev(u) = the smallest not-refused potential evictor (grows as evictors are refused;
final once that evictor is admitted, or INF).  k_b_async evaluates them with no barrier: every
wave owns a static slice of the round's work items and passes over its unsettled ones until none
is left, reading the other waves' states and eviction times as they happen to be -- possibly
stale.  This model runs the same rules item by item under a seeded random interleaving of waves,
with each read of another vertex's state / eviction time taken, at random, from an older snapshot
(a stale value is always an older value: states only move UND -> IN / OUT, eviction times only
grow), and colours whole graphs round by round.  tests/test_fold_model.py checks that the result
equals the oracle's variant B bit for bit: the claim "staleness delays a decision, never changes
it" that makes the GPU fold correct.
"""
import random

UND, IN, OUT = 0, 1, 2
INF = 0x7FFFFFFF


def _mex(s):
    m = 0
    while m in s:
        m += 1
    return m


def _seed_colouring(n, deg):
    """coloring_optimized.py:70-80 (as coloring.py:12-35): isolated vertices colour 0, then the
    uncoloured vertex of largest degree (ties -> last in file order) colour 0."""
    colour = [0 if deg[v] == 0 else -1 for v in range(n)]
    best = None
    for v in range(n):
        if colour[v] == -1 and (best is None or deg[v] >= deg[best]):
            best = v
    if best is not None:
        colour[best] = 0
    return colour


def fold_round(adj, deg, cand, U, rng, waves=5, stale=0.3, snap_every=3):
    """One round's fold over the proposers U (all uncoloured vertices, candidates cand) as the
    asynchronous waves evaluate it; returns the winners (admitted, never evicted)."""
    st = {v: UND for v in U}
    ev = {v: -1 for v in U}
    # row ranges: admission looks at earlier-or-later entries of degree >= deg(v) (only earlier
    # ones count), eviction at entries of higher degree (only later ones count)
    adm_rows = {v: [u for u in adj[v] if deg[u] >= deg[v]] for v in U}
    ev_rows = {v: [u for u in adj[v] if deg[u] > deg[v]] for v in U}
    cur = {v: 0 for v in U}
    snaps = [(dict(st), dict(ev))]

    def read_st(x):
        if x not in st:
            return OUT  # not a proposer this round: never same-candidate (coloured)
        return rng.choice(snaps)[0][x] if rng.random() < stale else st[x]

    def read_ev(x):
        return rng.choice(snaps)[1][x] if rng.random() < stale else ev[x]

    order = list(U)
    slices = [order[i * len(order) // waves:(i + 1) * len(order) // waves] for i in range(waves)]
    items = [[(v, "adm") for v in sl] for sl in slices]
    steps = 0
    while any(items):
        w = rng.choice([i for i in range(waves) if items[i]])
        v, kind = items[w].pop(0)
        keep = None
        if kind == "adm":
            c, refused, first = cand[v], False, None
            row = adm_rows[v]
            for i in range(cur[v], len(row)):
                u = row[i]
                f = 0
                if u < v and u in st and cand[u] == c:
                    su = read_st(u)
                    if su == UND:
                        f = 2
                    elif su == IN:
                        e = read_ev(u)
                        if e > v:
                            f = 1
                        elif e >= 0 and read_st(e) == IN:
                            f = 0
                        else:
                            f = 2
                if f == 1:
                    refused = True
                    break
                if f == 2 and first is None:
                    first = i
            if refused:
                st[v] = OUT
            elif first is not None:
                cur[v] = first
                keep = (v, "adm")
            else:
                st[v] = IN
                keep = (v, "ev")
        else:
            c = cand[v]
            e = INF
            for x in ev_rows[v]:
                if x > v and x in st and cand[x] == c and read_st(x) != OUT:
                    e = min(e, x)
            ev[v] = e
            if e != INF and read_st(e) != IN:
                keep = (v, "ev")
        if keep is not None:
            items[w].append(keep)
        steps += 1
        if steps % snap_every == 0:
            snaps.append((dict(st), dict(ev)))
            if len(snaps) > 6:
                snaps.pop(1)
        if steps > 200 * (len(U) + 1) ** 2:
            raise RuntimeError("the fold model does not converge")
    return [v for v in U if st[v] == IN and ev[v] == INF]


def model_color_b(rp, col, seed=0, waves=5, stale=0.3):
    """Variant B (coloring_optimized.py), unbounded, every round's fold by fold_round."""
    rng = random.Random(seed)
    n = len(rp) - 1
    adj = [[int(u) for u in col[rp[v]:rp[v + 1]]] for v in range(n)]
    deg = [len(a) for a in adj]
    colour = _seed_colouring(n, deg)
    rounds = 0
    while True:
        U = [v for v in range(n) if colour[v] == -1]
        if not U:
            return colour, rounds
        cand = {v: _mex({colour[u] for u in adj[v] if colour[u] >= 0}) for v in U}
        for v in fold_round(adj, deg, cand, U, rng, waves, stale):
            colour[v] = cand[v]
        rounds += 1
        if rounds > 4 * n + 16:
            raise RuntimeError("round limit")
