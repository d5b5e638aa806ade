"""bench.py's multi-GPU entry on the GPU box.

The driver measures N = 1, 2, 4, 8 with `bench.py --gpus N`; these run the N > 1 path on the
box's one GPU: two ranks started by bench.py itself (no outside launcher), both on GPU 0
over gloo (two processes cannot share one GPU in an RCCL group), and the one-rank RCCL
group (`--sharded` at N = 1).  Each line must carry the N it ran with, and the step on the
one-GPU step's definition; bench.py itself asserts the colouring equals the one-GPU engine's.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _bench(tmp_path, args, env_extra=None, timeout=600):
    out = tmp_path / "line.json"
    env = dict(os.environ, **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args + ["--json-out", str(out)],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return json.loads(out.read_text())


def test_bench_gpus2_spawns_two_ranks(tmp_path):
    line = _bench(tmp_path, ["--gpus", "2", "--workload", "rmat20", "--steps", "2", "--warmup", "1"],
                  {"GC_BENCH_BACKEND": "gloo", "GC_BENCH_DEVICE": "0"})
    assert line["n_gpus"] == 2 and line["steps"] == 2
    c = line["config"]
    assert c["multi"] == "hybrid" and c["switch_round"] is not None
    assert "validate_range" in c["step"] or "gc_validate_range" in c["step"]
    assert set(line["phases_ms"]) == {"create", "colour", "validate", "destroy"}
    assert c["single_gpu_ms"] > 0 and c["speedup_vs_single_gpu"] > 0 and c["hubs_on"]
    assert line["value"] > 0 and line["roofline"]["frac"] > 0


def test_bench_one_rank_rccl(tmp_path):
    line = _bench(tmp_path, ["--sharded", "--workload", "rmat20", "--steps", "2", "--warmup", "1"])
    assert line["n_gpus"] == 1 and "RCCL" in line["config"]["parallelism"]
    assert line["config"]["switch_round"] is not None

