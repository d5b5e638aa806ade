set -euo pipefail
mkdir -p gpurun_out/r02k
timeout -k 10 900 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_priority.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02k/pytest.log 2>&1 || { tail -40 gpurun_out/r02k/pytest.log; exit 1; }
tail -3 gpurun_out/r02k/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02k rmat24 - "GC_SWEEP_PAD=1" "GC_SWEEP_PAD=0"
STEPS=3 bash tools/gpu_ab.sh r02k rmat26 - "GC_SWEEP_PAD=1"
bash tools/gpu_trace_ab.sh r02k rmat26 -
