"""Host-compiled checks of device helpers (hipcc host code, no GPU): gc_deg_code, the monotone
byte code of a degree that the rank partition (csrc/gc_prep.hip, coloring.py:64's order)
gathers before the full degree (tests/host_code/deg_code.cpp)."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG_DIR, REPO


def test_deg_code_monotone_and_exact(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "deg_code")
    cmd = [hipcc, "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"), "-I", os.path.join(PKG_DIR, "csrc"),
           os.path.join(REPO, "tests", "host_code", "deg_code.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout[-2000:]
