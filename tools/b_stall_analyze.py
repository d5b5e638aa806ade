#!/usr/bin/env python3
"""What the asynchronous fold was waiting on when a k_b_async launch gave up (CPU analysis of a
GC_B_STALL_DUMP, tools/b_stall_probe.py).

The fold's convergence argument (csrc/gc_variant_b.hip, k_b_async): every wait of an admission
item v is on something EARLIER than v -- an earlier same-candidate neighbour u of degree >=
deg(v) that is still undecided, or admitted with an eviction time not yet known -- so the
earliest unsettled admission item can always settle.  This script takes the state the launch
left (states k8, candidates, eviction times ev, the listed items and their pending entries) on
the same graph (tests/golden/make_rmat_fixtures.py's numpy replica of the device generator) and,
for the earliest listed admission items, evaluates coloring_optimized.py's admission rule with
those states: what each one waits on, and whether that is itself listed (a real chain) or
already settled (the wave never saw the settled state: a visibility fault).
Usage: python tools/b_stall_analyze.py PREFIX SCALE SEED [K]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

INF = 0x7FFFFFFF
UND, IN, OUT = 0, 1, 2


def load(prefix, name, dtype):
    p = f"{prefix}.{name}.bin"
    return np.fromfile(p, dtype=dtype) if os.path.exists(p) else None


def main():
    prefix, scale, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    import make_rmat_fixtures as mk
    rp, col = mk.rmat_device_csr(scale, seed=seed)
    n = len(rp) - 1
    deg = np.diff(rp).astype(np.int64)
    info = open(f"{prefix}.info.txt").read().strip()
    k8 = load(prefix, "k8", np.uint8)
    cand_full = load(prefix, "cand", np.int32)
    ev = load(prefix, "ev", np.int32)
    adm = load(prefix, "adm", np.int32)
    heavy = load(prefix, "heavy", np.int32)
    evict = load(prefix, "evict", np.int32)
    state = (k8 & 3).astype(np.int64)
    c6 = (k8 >> 2).astype(np.int64)
    cand = np.where(c6 == 62, cand_full, c6)
    print(info)
    print(f"listed: {len(adm)} admissions, {len(heavy)} heavy admissions, {len(evict)} eviction times")
    listed_adm = set(adm.tolist()) | set(heavy.tolist())
    listed_ev = set(evict.tolist())
    # states of the listed items themselves (an admission item should be UND, an eviction item IN)
    bad_adm = [v for v in listed_adm if state[v] != UND]
    bad_ev = [v for v in listed_ev if state[v] != IN]
    print(f"listed admissions not UND: {len(bad_adm)}; listed eviction items not IN: {len(bad_ev)}")
    # UND proposers that no list holds (every uncoloured vertex proposes in variant B)
    und = np.nonzero((state == UND) & (c6 != 63))[0]
    orphan = [int(v) for v in und if int(v) not in listed_adm]
    print(f"UND proposers: {len(und)}; not listed: {len(orphan)} (first {orphan[:10]})")
    order = sorted(listed_adm)
    for v in order[:K]:
        cv = int(cand[v])
        nb = col[rp[v]:rp[v + 1]]
        rng = nb[(nb < v) & (deg[nb] >= deg[v])]
        rng = rng[(cand[rng] == cv) & (state[rng] != OUT) & (c6[rng] != 63)]
        waits = []
        verdict = "admit"
        for u in sorted(set(rng.tolist())):
            su = int(state[u])
            if su == UND:
                waits.append(f"u={u} UND ({'listed' if u in listed_adm else 'NOT listed'})")
                verdict = "wait"
            else:  # IN
                e = int(ev[u])
                if e == INF or e > v:
                    if e != INF and state[e] == UND:
                        waits.append(f"u={u} IN ev={e}>v (refuses)")
                    else:
                        waits.append(f"u={u} IN ev={'INF' if e == INF else e} (refuses)")
                    verdict = "refused"
                    break
                if e >= 0 and state[e] == IN:
                    continue  # evicted before v arrived
                waits.append(f"u={u} IN ev={e} state(ev)={int(state[e]) if e >= 0 else '-'} "
                             f"(eviction item {'listed' if u in listed_ev else 'NOT listed'})")
                verdict = "wait" if verdict == "admit" else verdict
        print(f"item v={v} deg={deg[v]} cand={cv}: {verdict}; {len(rng)} entries in range; " + "; ".join(waits[:6]))


if __name__ == "__main__":
    main()
