set -euo pipefail
# BIGROW 2048 + parallel close reads: whole GPU suite, then R-MAT-24 / mesh / C2 benches
T=r02v21; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - -
STEPS=5 bash tools/gpu_ab.sh $T mesh512 -
STEPS=10 bash tools/gpu_ab.sh $T uniform10M -
