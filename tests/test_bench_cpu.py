"""bench.py's host logic (no GPU): the N-GPU workload scaling, the PMC summaries' build
identity (a summary of another libgcolor.so is never used), the roofline's capped credit."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_scaled_workload_weak_and_strong():
    w = bench.WORKLOADS["rmat24"]
    assert bench.scaled_workload(w, 1, "weak")["scale"] == 24
    assert bench.scaled_workload(w, 8, "weak")["scale"] == 27
    assert bench.scaled_workload(w, 8, "strong")["scale"] == 24
    assert "x 8 GPUs" in bench.scaled_workload(w, 8, "weak")["desc"]
    assert bench.scaled_workload(bench.WORKLOADS["uniform10M"], 4, "weak")["n"] == 40_000_000
    assert bench.scaled_workload(bench.WORKLOADS["mesh512"], 2, "weak")["dims"] == (512, 512, 1024)
    assert w["scale"] == 24  # the table is not modified


def test_pmc_summary_of_another_build_is_stale(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    os.makedirs(tmp_path / "profiles" / "pmc")
    p = tmp_path / "profiles" / "pmc" / "rmat24.json"
    per = {"k_commit": {"launches": 10, "hbm_bytes_per_launch": 100.0},
           "_step": {"steps": 1, "bytes": 8e12}}
    monkeypatch.setattr(bench, "lib_sha16", lambda: "abc")
    p.write_text(json.dumps(dict(per, _build="other")))
    assert bench.pmc_class_bytes("rmat24", "A")[0] == {}
    assert "stale" in bench.pmc_class_bytes("rmat24", "A")[1]
    assert bench.pmc_step_frac("rmat24", "A", 1.0) is None
    p.write_text(json.dumps(dict(per, _build="abc")))
    cls, src = bench.pmc_class_bytes("rmat24", "A")
    assert cls["commit"] == 100.0 and "stale" not in src
    assert abs(bench.pmc_step_frac("rmat24", "A", 1.0)["frac"] - 1.0) < 1e-12


def test_capped_credit():
    kern = {"propose": {"bytes": 1e12, "ms": 10.0, "launches": 1}, "commit": {"bytes": 1e9, "ms": 10.0, "launches": 1}}
    cap = bench.capped_alg(kern, n=0, nnz=0)
    assert cap == 10e-3 * bench.HBM_PEAK_GBS * 1e9 + 1e9


def test_replica_workload():
    w = bench.WORKLOADS["rmat24"]
    r3 = bench.replica_workload(w, 8, 3)
    assert r3["scale"] == 24 and r3["seed"] == w["seed"] + 3 and "8 independent colourings" in r3["desc"]
    assert bench.replica_workload(bench.WORKLOADS["mesh512"], 4, 2)["dims"] == (512, 512, 512)
    assert w["seed"] == 1  # the table is not modified


def test_bench_rejects_mismatched_world():
    """Under a launcher, --gpus must equal the ranks started (the flag was ignored and
    an un-launched N > 1 run printed n_gpus 1).  Checked before anything touches a GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(bench.REPO, "bench.py"), "--gpus", "2"], cwd=bench.REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_spawn_ranks_command(monkeypatch):
    """`bench.py --gpus N` without WORLD_SIZE starts torch.distributed.run with N ranks on
    127.0.0.1 as a child process (never an exec) and returns its status."""
    import subprocess
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    assert bench.spawn_ranks(4) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "3"][-4:]


def test_calibrated_fractions(tmp_path, monkeypatch):
    """The calibrated physical basis (2 x FETCH_SIZE + WRITE_SIZE: FETCH_SIZE counts half of
    every line read, profiles/calib/gather_bytes.json) in the step fraction and the dominant
    class's roofline; the calibration itself is the committed measurement."""
    cal = bench.calibration()
    assert cal and cal["fetch_counted_over_streamed_bytes"] == 0.5
    assert 60 <= cal["fetch_counted_per_random_gather_B"] <= 68 and cal["gather_Gops"] > 10
    calib_src = os.path.join(bench.REPO, "profiles", "calib", "gather_bytes.json")
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    os.makedirs(tmp_path / "profiles" / "pmc")
    os.makedirs(tmp_path / "profiles" / "calib")
    (tmp_path / "profiles" / "calib" / "gather_bytes.json").write_text(open(calib_src).read())
    monkeypatch.setattr(bench, "lib_sha16", lambda: "abc")
    per = {"k_sweep_async": {"launches": 4, "hbm_bytes_per_launch": 3e6, "hbm_bytes_per_launch_calibrated": 5e6},
           "_step": {"steps": 1, "bytes": 3e9, "fetch_bytes": 2e9, "write_bytes": 1e9}, "_build": "abc"}
    (tmp_path / "profiles" / "pmc" / "rmat26.json").write_text(json.dumps(per))
    f = bench.pmc_step_frac("rmat26", "A", 1.0)
    assert f["bytes_per_step_calibrated"] == 5e9 and abs(f["frac_calibrated"] - 5.0 / bench.HBM_PEAK_GBS) < 1e-12
    kern = {"sweep": {"ms": 2.0, "launches": 4, "bytes": 0.0}, "propose": {"ms": 1.0, "launches": 4, "bytes": 1.0}}
    r = bench.calibrated_roofline("rmat26", "A", kern)
    assert r["kernel"] == "sweep" and r["traffic"] == 5e6
    assert abs(r["achieved"] - 5e6 / 0.5e-3 / 1e9) < 1e-9
    assert abs(r["frac_of_gather_ceiling"] - r["achieved"] / cal["gather_ceiling_GBps"]) < 1e-12
