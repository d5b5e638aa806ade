set -euo pipefail
mkdir -p gpurun_out/r02zk
B=$(pwd)/build_variants
STEPS=3 bash tools/gpu_ab.sh r02zk rmat24 - "GC_LIB_PATH=$B/t512/libgcolor.so" "GC_LIB_PATH=$B/t2k/libgcolor.so" "GC_LIB_PATH=$B/t4k/libgcolor.so" "GC_TAIL_HMAX_HUB=64" "GC_TAIL_HMAX_HUB=192" -
STEPS=2 bash tools/gpu_ab.sh r02zk rmat26 - "GC_LIB_PATH=$B/t2k/libgcolor.so" "GC_LIB_PATH=$B/t4k/libgcolor.so" -
