set -euo pipefail
# new grid defaults: GPU suite + benches
T=r02v24; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - - "GC_GRID_PS=1024 GC_GRID_S=384"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 -
STEPS=5 bash tools/gpu_ab.sh $T mesh512 -
STEPS=10 bash tools/gpu_ab.sh $T uniform10M - "GC_GRID_PS=1024 GC_GRID_S=384"
