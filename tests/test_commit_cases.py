"""The k_commit corner-case states of tests/commit_cases.py, checked on CPU against the numpy
restatement of the round loop (tests/shard_numpy.py, the stand-in for gc_color_resume): the
expected colours and records the GPU tests assert are the reference's."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from commit_cases import stage_overflow_case, stage_overflow_tree  # noqa: E402
from shard_numpy import numpy_resume  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402


@pytest.mark.parametrize("K,leaves,n", [(8, 3, 40), (64, 9, 1000), (130, 40, 6000)])
def test_stage_overflow_case_expectation(K, leaves, n):
    rp, col, colors, front, exp = stage_overflow_case(K, leaves, n)
    assert np.array_equal(np.diff(rp)[:K], np.full(K, leaves + 1))
    res = numpy_resume(rp, col)(torch.from_numpy(colors), None, torch.from_numpy(front), 3, None, True, True, True)
    assert res.status == 0
    assert np.array_equal(res.colors, exp["colors"])
    assert list(res.round_F[:2]) == exp["F"] and list(res.round_accepted[:2]) == exp["accepted"]
    assert list(res.round_U[:2]) == exp["U"]
    assert tuple(oracle.c_validate(rp, col, res.colors)) == (0, 0)


@pytest.mark.parametrize("fanout,levels,n", [(3, 4, 100), (5, 5, 5000), (61, 4, 300_000)])
def test_stage_overflow_tree_expectation(fanout, levels, n):
    rp, col, exp = stage_overflow_tree(fanout, levels, n)
    deg = np.diff(rp)
    assert deg[0] == fanout + 2 and deg.max() == fanout + 2 and (deg[1:] <= fanout + 1).all()
    o = oracle.c_color(rp, col, "A")
    assert o["status"] == 0 and np.array_equal(o["colors"], exp["colors"])
    assert list(o["round_F"][:-1]) == exp["F"] and list(o["round_accepted"][:-1]) == exp["F"]
    assert o["reseeds"] == 0
