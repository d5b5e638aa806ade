"""How the proposals of an R-MAT colouring spread over its rounds (CPU, no GPU needed).

Colours numpy R-MAT graphs (tests/test_oracle_omp.rmat_csr: the same (0.57, 0.19, 0.19) process
as the device generator, not the same stream) with the multi-core restatement
oracle/gcolor_omp.c and reports, per frontier threshold, how many rounds reach it and what share
of all proposals they hold.  This is the evidence behind DESIGN §7: most rounds are small
(latency-bound, nothing to shard), a few big rounds hold most of the proposals.

    python tools/round_structure.py 20 22 24 > profiles/r03/round_structure.txt
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT]
from test_oracle_omp import rmat_csr  # noqa: E402

from oracle import oracle  # noqa: E402


def main(scales):
    for scale in scales:
        t = time.time()
        rp, col = rmat_csr(scale, 16, 1)
        tg = time.time() - t
        n = len(rp) - 1
        t = time.time()
        o = oracle.omp_color(rp, col, symmetric=True, threads=min(16, os.cpu_count() or 1))
        tc = time.time() - t
        F = np.asarray(o["round_F"], np.int64)
        print(f"R-MAT-{scale} (numpy, seed 1): n={n} nnz={len(col)}  generated {tg:.0f} s, coloured {tc:.1f} s; "
              f"{len(F)} rounds, {o['max_color'] + 1} colours, {F.sum()} proposals")
        for thr in sorted({256, 1024, 4096, 16384, 65536, max(n // 64, 1)}):
            big = F >= thr
            print(f"  frontier >= {thr:>9}: {int(big.sum()):5d} rounds hold {F[big].sum() / max(F.sum(), 1):6.1%} of the "
                  f"proposals; {int((~big).sum()):5d} rounds below")
        q = np.percentile(F, [50, 75, 90, 99]).astype(int)
        print(f"  frontier percentiles 50/75/90/99: {q[0]} {q[1]} {q[2]} {q[3]}; max {int(F.max())}")
        sys.stdout.flush()
        del rp, col, o


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [20, 22])
