set -euo pipefail
# k_commit_big closes the round: GPU suite + A/B against a separate k_close (GC_TICKET_CLOSE=0)
T=r02v10; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_TICKET_CLOSE=0" - "GC_TICKET_CLOSE=0"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_TICKET_CLOSE=0"
