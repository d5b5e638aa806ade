"""The round close (csrc/gc_close.h) on the CPU: the batched form GC_CLOSE_BATCH builds use
(every control word loaded before any store) against the interleaved form of rounds 1-3, on
random control blocks, pre-read counters, modes and record positions (tests/host_close/
close_eq.hip, hipcc host code: __host__ __device__ functions, no GPU).  Both must leave the
same control block and the same round records (coloring.py:86-95, 110-132 as the engine
records them)."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG_DIR, REPO


@pytest.fixture(scope="module")
def close_eq(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    exe = str(tmp_path_factory.mktemp("close") / "close_eq")
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(PKG_DIR, "csrc"), os.path.join(REPO, "tests", "host_close", "close_eq.hip"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_batched_close_equals_interleaved(close_eq, seed):
    r = subprocess.run([close_eq, "300000", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok 300000", r.stdout[-2000:] + r.stderr[-2000:]
