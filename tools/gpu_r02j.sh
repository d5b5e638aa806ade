set -euo pipefail
mkdir -p gpurun_out/r02j
timeout -k 10 900 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02j/pytest.log 2>&1 || { tail -40 gpurun_out/r02j/pytest.log; exit 1; }
tail -3 gpurun_out/r02j/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02j rmat24 - "GC_SWEEP_LOOP=0"
STEPS=3 bash tools/gpu_ab.sh r02j rmat26 - "GC_SWEEP_LOOP=0"
STEPS=5 bash tools/gpu_ab.sh r02j uniform10M - "GC_SWEEP_LOOP=0"
bash tools/gpu_trace_ab.sh r02j rmat26 -
