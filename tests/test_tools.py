"""tools/round_cost.py's trace analysis on a synthetic kernel trace (CPU): the rounds are split
at their closing kernels and attributed to frontier-size classes as the GPU session expects."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, rounds, closing):
    """k_init ... INIT commit, then per round the kernels of `closing`'s pattern, k_finalize."""
    t = 1000
    rows = []

    def k(name, dur):
        nonlocal t
        rows.append({"Kernel_Name": f"{name}(GDev, GLists)", "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 500  # 0.5 us gap

    # an earlier colouring in the same trace: ignored (the analysis takes the last one)
    k("k_init", 9000)
    k("k_finalize", 100)
    k("k_init", 9000)
    k("k_seed_prep", 100)
    k("k_commit", 2000)
    k("k_commit_big", 100)
    k("k_close", 100)
    for r in range(rounds):
        k("k_propose", 3000 + 10 * r)
        k("k_resolve", 2000)
        k("k_sweep_async", 4000)
        if closing == "close":
            k("k_commit", 5000)
            k("k_commit_big", 1000)
            k("k_close", 2000)
        else:  # the ticket-closing commit (meshes, uniform graphs)
            k("k_commit", 6000)
    k("k_finalize", 100)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def _run(tmp_path, closing):
    F = [100, 2000, 30000, 70000, 500, 0]  # the last record: U == 0
    tr, rec = tmp_path / "trace.csv", tmp_path / "rec.json"
    _trace(tr, len(F) - 1, closing)
    rec.write_text(json.dumps({"workload": "synthetic", "F": F, "U": [1] * len(F), "accepted": [1] * len(F),
                               "seeds": [0] * len(F), "device_ms": 1.0}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "round_cost.py"), "analyze", str(tr), str(rec)],
                         check=True, capture_output=True, text=True).stdout
    return out


def test_round_cost_split_with_k_close(tmp_path):
    out = _run(tmp_path, "close")
    assert "comparing 5 rounds" in out
    # classes: [0,1024): F=100, 500; [1024,16384): 2000; [16384,65536): 30000; [65536,inf): 70000
    assert "F in [0, 1024): 2 rounds" in out
    assert "F in [1024, 16384): 1 rounds" in out
    assert "F in [65536, inf): 1 rounds" in out
    # one round: propose 3.0x + resolve 2 + sweep 4 + commit 5 + big 1 + close 2 us busy, 5 gaps of 0.5 us
    line = [ln for ln in out.splitlines() if ln.startswith("  F in [1024, 16384)")][0]
    assert "busy 17.0 + gaps 2.5" in line
    assert "k_close" in out and "k_sweep_async" in out


def test_round_cost_split_with_ticket_close(tmp_path):
    out = _run(tmp_path, "ticket")
    assert "comparing 5 rounds" in out
    line = [ln for ln in out.splitlines() if ln.startswith("  F in [1024, 16384)")][0]
    assert "busy 15.0 + gaps 1.5" in line
