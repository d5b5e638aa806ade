set -euo pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 900 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e/pytest.log 2>&1 || { tail -40 gpurun_out/r02e/pytest.log; exit 1; }
tail -3 gpurun_out/r02e/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02e rmat24 - "GC_HUB_SCAN=0"
STEPS=3 bash tools/gpu_ab.sh r02e rmat26 - "GC_HUB_SCAN=0" "GC_TAIL_HMAX_HUB=128"
bash tools/gpu_trace_ab.sh r02e rmat26 -
