set -euo pipefail
# undecided hub lists of hub indices: hub / parity / shard / full-size tests, A/B against the previous build
T=r02v35; mkdir -p gpurun_out/$T
B=$(pwd)/build_variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_LIB_PATH=$B/prev/libgcolor.so" - "GC_LIB_PATH=$B/prev/libgcolor.so"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_LIB_PATH=$B/prev/libgcolor.so"
