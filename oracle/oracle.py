"""Parity oracle: CPU restatements of the reference's colouring hot path.

TEST INFRASTRUCTURE / CHECKER ONLY -- importable from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, never from the product package.

Two independent restatements of the same semantics (see gcolor_oracle.c's header for
the reference file:line map, SURVEY.md §8a for the derivation):

* ``py_color``  -- pure-Python loops, written to mirror the reference's structure
  (coloring.py:73-132 / coloring_optimized.py:70-146) step by step; small graphs only.
* ``c_color``   -- the C restatement in gcolor_oracle.c via ctypes (fast; CPU baseline).

Parity is pinned: tests/test_oracle_golden.py checks both against the golden vectors
that tests/golden/make_golden.py recorded by executing the reference's own code.

Graphs are CSR over file positions: ``rp`` int64[n+1], ``col`` int32[nnz]; the
adjacency lists are kept exactly as listed (duplicates, self-loops, asymmetry).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libgcolor_oracle.so")

OK, FAILED, STALLED = 0, 1, 2


class _Summary(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_int64), ("fail_round", ctypes.c_int64),
                ("fail_count", ctypes.c_int64), ("reseeds", ctypes.c_int64),
                ("max_color", ctypes.c_int64), ("balg_propose", ctypes.c_double),
                ("balg_resolve", ctypes.c_double), ("balg_push", ctypes.c_double),
                ("balg_validate", ctypes.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        lib.oracle_color.argtypes = [P, P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                     P, P, P, P, P, P, P, ctypes.c_int64, ctypes.POINTER(_Summary)]
        lib.oracle_color.restype = ctypes.c_int
        lib.oracle_color_prio.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_uint64, ctypes.c_int32, P, P, P, P, P, P, P, ctypes.c_int64,
                                          ctypes.POINTER(_Summary)]
        lib.oracle_color_prio.restype = ctypes.c_int
        lib.prio_hash.argtypes = [ctypes.c_uint64, ctypes.c_int64]
        lib.prio_hash.restype = ctypes.c_uint32
        lib.oracle_validate.argtypes = [P, P, ctypes.c_int64, P, ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int64)]
        lib.oracle_validate.restype = None
        _lib = lib
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def c_color(rp, col, variant="A", k=None, e1=True, max_rounds=1 << 16):
    """Run the C restatement. ``k=None`` = unbounded. Returns a dict of numpy arrays."""
    lib = load()
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    n = rp.shape[0] - 1
    color = np.empty(n, np.int32)
    cround = np.empty(n, np.int32)
    per = {key: np.zeros(max_rounds, np.int64) for key in ("U", "F", "maxmex", "accepted", "seeds")}
    s = _Summary()
    st = lib.oracle_color(_ptr(rp), _ptr(col), n, 0 if variant == "A" else 1, -1 if k is None else int(k),
                          1 if e1 else 0, _ptr(color), _ptr(cround), _ptr(per["U"]), _ptr(per["F"]),
                          _ptr(per["maxmex"]), _ptr(per["accepted"]), _ptr(per["seeds"]), max_rounds,
                          ctypes.byref(s))
    if st < 0:
        raise RuntimeError(f"oracle_color failed with status {st}")
    r = s.rounds
    out = {"status": st, "colors": color, "colored_round": cround, "rounds": r,
           "fail_round": s.fail_round, "fail_count": s.fail_count, "reseeds": s.reseeds,
           "max_color": s.max_color,
           "balg": {"propose": s.balg_propose, "resolve": s.balg_resolve, "push": s.balg_push,
                    "validate": s.balg_validate}}
    for key, arr in per.items():
        out["round_" + key] = arr[:r].copy()
    return out


_omp = None
OMP_LIB_PATH = os.path.join(HERE, "build", "libgcolor_omp.so")


def load_omp():
    global _omp
    if _omp is None:
        if not os.path.exists(OMP_LIB_PATH):
            build()
        lib = ctypes.CDLL(OMP_LIB_PATH)
        P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.omp_color.argtypes = [P, P, I64, I32, I32, P, P, P, P, P, P, P, I64, ctypes.POINTER(I64),
                                  ctypes.POINTER(I64)]
        lib.omp_color.restype = ctypes.c_int
        _omp = lib
    return _omp


def omp_color(rp, col, symmetric=False, threads=0, want_rounds=True, max_rounds=1 << 17):
    """The multi-core C restatement (gcolor_omp.c, variant A, unbounded, E1 on): the CPU
    baseline of bench.py.  threads=0: OpenMP's default (OMP_NUM_THREADS / all cores)."""
    lib = load_omp()
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    n = rp.shape[0] - 1
    color = np.empty(max(n, 1), np.int32)
    cround = np.empty(max(n, 1), np.int32) if want_rounds else None
    cap = max_rounds if want_rounds else 0
    per = {key: np.zeros(max(cap, 1), np.int64) for key in ("U", "F", "maxmex", "accepted", "seeds")}
    rounds, reseeds = ctypes.c_int64(), ctypes.c_int64()
    pp = (lambda a: _ptr(a)) if want_rounds else (lambda a: None)
    st = lib.omp_color(_ptr(rp), _ptr(col), n, 1 if symmetric else 0, int(threads), _ptr(color),
                       None if cround is None else _ptr(cround), pp(per["U"]), pp(per["F"]), pp(per["maxmex"]),
                       pp(per["accepted"]), pp(per["seeds"]), cap, ctypes.byref(rounds), ctypes.byref(reseeds))
    if st < 0:
        raise RuntimeError(f"omp_color failed with status {st}")
    r = rounds.value
    out = {"status": st, "colors": color[:n], "colored_round": None if cround is None else cround[:n],
           "rounds": r, "reseeds": reseeds.value, "max_color": int(color[:n].max()) if n else -1}
    if want_rounds:
        for key, arr in per.items():
            out["round_" + key] = arr[:r].copy()
    return out


def c_color_prio(rp, col, k=None, e1=True, priority=1, seed=0, speculative=False, max_rounds=1 << 16):
    """Variant A with seeded priorities (priority=1: rank (prio_hash(seed, v), pos) in the
    per-colour LFMIS) and/or speculative first-fit rounds with one-shot resolution."""
    lib = load()
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    n = rp.shape[0] - 1
    color = np.empty(max(n, 1), np.int32)
    cround = np.empty(max(n, 1), np.int32)
    per = {key: np.zeros(max_rounds, np.int64) for key in ("U", "F", "maxmex", "accepted", "seeds")}
    s = _Summary()
    st = lib.oracle_color_prio(_ptr(rp), _ptr(col), n, -1 if k is None else int(k), 1 if e1 else 0, int(priority),
                               int(seed) & (2**64 - 1), 1 if speculative else 0, _ptr(color), _ptr(cround),
                               _ptr(per["U"]), _ptr(per["F"]), _ptr(per["maxmex"]), _ptr(per["accepted"]),
                               _ptr(per["seeds"]), max_rounds, ctypes.byref(s))
    if st < 0:
        raise RuntimeError(f"oracle_color_prio failed with status {st}")
    r = s.rounds
    out = {"status": st, "colors": color[:n], "colored_round": cround[:n], "rounds": r,
           "fail_round": s.fail_round, "fail_count": s.fail_count, "reseeds": s.reseeds,
           "max_color": s.max_color}
    for key, arr in per.items():
        out["round_" + key] = arr[:r].copy()
    return out


def prio_hash(seed, v):
    return load().prio_hash(int(seed) & (2**64 - 1), int(v))


def c_validate(rp, col, colors):
    lib = load()
    rp = np.ascontiguousarray(rp, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    colors = np.ascontiguousarray(colors, dtype=np.int32)
    u, c = ctypes.c_int64(), ctypes.c_int64()
    lib.oracle_validate(_ptr(rp), _ptr(col), rp.shape[0] - 1, _ptr(colors), ctypes.byref(u), ctypes.byref(c))
    return u.value, c.value


# ------------------------------------------------------------------------------------------
# pure-Python restatement (mirrors the reference's control flow; small graphs only)
# ------------------------------------------------------------------------------------------

def _components_argmax(adj, deg, color):
    """E1 helper: argmax-(deg,pos) vertex of each component of the uncoloured subgraph."""
    n = len(adj)
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for v in range(n):
        if color[v] != -1:
            continue
        for u in adj[v]:
            if color[u] == -1:
                a, b = find(v), find(u)
                if a != b:
                    parent[max(a, b)] = min(a, b)
    best = {}
    for v in range(n):
        if color[v] == -1:
            r = find(v)
            if r not in best or deg[v] >= deg[best[r]]:
                best[r] = v
    return sorted(best.values())


def py_prio_hash(seed, v):
    """Pure-Python prio_hash (splitmix64 finaliser, top 32 bits) -- checks the C one."""
    M = (1 << 64) - 1
    z = (int(seed) + 0x9E3779B97F4A7C15 * (v + 1)) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    z ^= z >> 31
    return z >> 32


def py_color(adj, variant="A", k=None, e1=True, priority_seed=None, speculative=False):
    """Pure-Python restatement. ``adj`` = list of neighbour-position lists (file order).
    ``priority_seed``: sort each candidate group by py_prio_hash(seed, v) instead of deg
    (coloring.py:64's key); ``speculative``: every uncoloured vertex proposes and keeps its
    proposal iff no listed lower-rank neighbour proposed the same colour (variant A)."""
    n = len(adj)
    deg = [len(a) for a in adj]
    rkey = deg if priority_seed is None else [py_prio_hash(priority_seed, v) for v in range(n)]
    kk = None if k is None else int(k)
    # coloring.py:12-17
    color = [0 if deg[v] == 0 else -1 for v in range(n)]
    cround = [0 if color[v] == 0 else -1 for v in range(n)]
    # coloring.py:19-35 -- left fold: x if len(x) > len(y) else y  => last maximum
    seed = None
    for v in range(n):
        if color[v] == -1 and (seed is None or not (deg[seed] > deg[v])):
            seed = v
    if seed is not None:
        color[seed] = 0
        cround[seed] = 0
    rounds_U, rounds_F, rounds_maxmex = [], [], []
    status, fail_round, fail_count, reseeds = OK, -1, 0, 0
    r = 0
    while True:
        U = [v for v in range(n) if color[v] == -1]          # coloring.py:86-88
        rounds_U.append(len(U))
        if not U:
            rounds_F.append(0)
            rounds_maxmex.append(-1)
            break
        props = []                                            # (cand, v) in file order
        fails = 0
        for v in U:                                           # coloring.py:98-102
            used = set(color[u] for u in adj[v] if color[u] != -1)
            if not used:
                if variant == "A" and not speculative:
                    continue                                  # -2
                if speculative and kk is not None and kk <= 0:
                    fails += 1
                props.append((0, v))                          # coloring_optimized.py:159-160
                continue
            c = 0
            while c in used:
                c += 1
            if kk is not None and c >= kk:
                fails += 1                                    # -3
            props.append((c, v))
        rounds_F.append(len(props))
        rounds_maxmex.append(max((c for c, _ in props), default=-1))
        if fails:                                             # coloring.py:104-108
            status, fail_round, fail_count = FAILED, r, fails
            break
        if not props:                                         # stall (coloring.py:93-95) -> E1
            if not e1:
                status = STALLED
                break
            for s in _components_argmax(adj, deg, color):
                color[s] = 0
                cround[s] = r + 1
                reseeds += 1
            r += 1
            continue
        groups = {}
        for c, v in props:                                    # groupByKey, file order
            groups.setdefault(c, []).append(v)
        accepted = []
        for c, members in groups.items():
            if speculative:                                   # one-shot: lower-rank same-colour proposer loses v
                mem = set(members)
                for v in members:
                    if not any(u in mem and (rkey[u], u) < (rkey[v], v) for u in adj[v]):
                        accepted.append((v, c))
            elif variant == "A":                              # coloring.py:56-70
                taken = set()
                for v in sorted(members, key=lambda x: rkey[x]):
                    if not any(u in taken for u in adj[v]):
                        taken.add(v)
                        accepted.append((v, c))
            else:                                             # coloring_optimized.py:168-184
                acc = []
                for v in members:
                    cand_list = sorted(acc + [v], key=lambda x: deg[x], reverse=True)
                    taken, res = set(), []
                    for x in cand_list:
                        if not any(u in taken for u in adj[x]):
                            taken.add(x)
                            res.append(x)
                    acc = res
                accepted.extend((v, c) for v in acc)
        for v, c in accepted:                                 # coloring.py:117-127
            color[v] = c
            cround[v] = r + 1
        r += 1
    return {"status": status, "colors": color, "colored_round": cround, "round_U": rounds_U,
            "round_F": rounds_F, "round_maxmex": rounds_maxmex, "fail_round": fail_round,
            "fail_count": fail_count, "reseeds": reseeds,
            "max_color": max(color) if color else -1}


def py_validate(adj, colors):
    """coloring.py:149-162 counts."""
    unc = sum(1 for c in colors if c == -1)
    conf = sum(1 for v, a in enumerate(adj) for u in a if colors[u] == colors[v])
    return unc, conf
