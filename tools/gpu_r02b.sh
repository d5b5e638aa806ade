set -euo pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1 || { tail -40 gpurun_out/r02b/pytest.log; exit 1; }
tail -3 gpurun_out/r02b/pytest.log
bash tools/gpu_ab.sh r02b rmat24 - "GC_HUB_CHUNK=0" "GC_TAIL_HMAX_HUB=256" "GC_TAIL_HMAX_HUB=1024"
bash tools/gpu_ab.sh r02b rmat26 - "GC_HUB_CHUNK=0" "GC_TAIL_HMAX_HUB=256" "GC_TAIL_HMAX_HUB=1024"
