set -euo pipefail
# A/B: per-wave flush of the undecided list in JP sweeps over short lists
T=r02v14; mkdir -p gpurun_out/$T
B=$(pwd)/build_variants
GC_LIB_PATH=$B/wf64k/libgcolor.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_LIB_PATH=$B/wf4k/libgcolor.so" "GC_LIB_PATH=$B/wf64k/libgcolor.so" - "GC_LIB_PATH=$B/wf4k/libgcolor.so" "GC_LIB_PATH=$B/wf64k/libgcolor.so"
