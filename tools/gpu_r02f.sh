set -euo pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 900 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_priority.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02f/pytest.log 2>&1 || { tail -40 gpurun_out/r02f/pytest.log; exit 1; }
tail -3 gpurun_out/r02f/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02f rmat24 - "GC_TAIL_HMAX_HUB=128"
STEPS=3 bash tools/gpu_ab.sh r02f rmat26 - "GC_TAIL_HMAX_HUB=128"
bash tools/gpu_trace_ab.sh r02f rmat26 -
