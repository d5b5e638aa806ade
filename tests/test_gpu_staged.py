"""Staged GPU tests (marker gpu_staged, NOT selected by -m gpu): opt-in paths not yet timed on
the GPU, run with `pytest -m gpu_staged` and promoted to `gpu` (switched on) or removed once
measured.
Run: GC_RUN_STAGED=1 python -m pytest tests/test_gpu_staged.py -m gpu_staged -x -v [-k GROUP]

* validate_c8: the validation from the byte mirror (GC_VALIDATE_C8=1).

Round 4 measured and removed the other round-3 paths (profiles/r04/c): variant B's asynchronous
fold (GC_B_ASYNC), the asynchronous JP on hub-less graphs (GC_ASYNC=2), the first sweep inside
k_sweep_async (GC_ASYNC_RESOLVE), k_commit_big closing the round (GC_BIG_CLOSE), hipGraph
replay of the rounds (GC_GRAPHS) and capped small-round grids (GC_GRID_SMALL): each was
bit-exact (profiles/r04/b) and slower or within noise.  The resume / hybrid / stage-overflow
tests moved to tests/test_gpu_resume.py.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

# selected only by `-m gpu_staged` with GC_RUN_STAGED=1 (the CPU suite's -m "not gpu" skips them)
pytestmark = [pytest.mark.gpu_staged,
              pytest.mark.skipif(not os.environ.get("GC_RUN_STAGED"), reason="staged: GC_RUN_STAGED=1 -m gpu_staged")]


# --- validation from the byte mirror (GC_VALIDATE_C8=1, the resident colouring) -------------
def test_validate_c8_matches(monkeypatch):
    """The resident colouring validated from c8 counts what the int colours count: after a full
    run, after a failed bounded run (uncoloured vertices), and after a resume from a state with
    planted conflicts (colours < 254 and >= 254, the byte mirror's BIG case)."""
    import torch
    from gcolor_amd.engine import DeviceGraph
    with DeviceGraph.rmat(12, 16, seed=9) as dg:
        rp, col = dg.export()
        for k in (None, 3):
            g = dg.color("A", num_colors=k)
            monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
            ref = dg.validate()
            monkeypatch.setenv("GC_VALIDATE_C8", "1")
            assert dg.validate() == ref == tuple(oracle.c_validate(rp, col, g.colors))
        v = int(np.argmax(np.diff(rp)))  # the largest row: it has neighbours
        u = int(col[rp[v]])
        c = np.full(dg.n, -1, np.int32)
        c[v], c[u] = 300, 300  # a conflict past the byte mirror
        w = next(int(x) for x in col[rp[u]:rp[u + 1]] if int(x) not in (u, v))
        x = next((int(y) for y in col[rp[w]:rp[w + 1]] if int(y) not in (u, v, w)), None)
        c[w] = 5
        if x is not None:
            c[x] = 5  # a conflict below 254
        front = np.array(sorted(y for y in set(int(y) for y in col[rp[v]:rp[v + 1]]) if c[y] < 0), np.int32)
        ct, ft = torch.from_numpy(c).cuda(), torch.from_numpy(front if len(front) else np.zeros(1, np.int32)).cuda()
        torch.cuda.synchronize()
        g = dg.resume(ct.data_ptr(), ft.data_ptr(), len(front), 0)
        monkeypatch.delenv("GC_VALIDATE_C8", raising=False)
        ref = dg.validate()
        monkeypatch.setenv("GC_VALIDATE_C8", "1")
        assert dg.validate() == ref == tuple(oracle.c_validate(rp, col, g.colors))
        assert ref[1] > 0

