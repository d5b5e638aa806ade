set -euo pipefail
# sweeps without stats (default now): parity; A/B per-wave stats atomics in the other round kernels
T=r02v13; mkdir -p gpurun_out/$T
B=$(pwd)/build_variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubs.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_LIB_PATH=$B/statwave/libgcolor.so" - "GC_LIB_PATH=$B/statwave/libgcolor.so"
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - "GC_LIB_PATH=$B/statwave/libgcolor.so"
STEPS=10 bash tools/gpu_ab.sh $T uniform10M - "GC_LIB_PATH=$B/statwave/libgcolor.so"
