set -euo pipefail
mkdir -p gpurun_out/r02zf
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zf/pytest.log 2>&1 || { tail -30 gpurun_out/r02zf/pytest.log; exit 1; }
tail -2 gpurun_out/r02zf/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02zf rmat24 - "GC_GRID_S=1024"
