set -euo pipefail
# vertices per wave chunk capped at 32 / 16 (big rounds: shorter long poles?)
T=r02v41; mkdir -p gpurun_out/$T
B=$(pwd)/build_variants
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_LIB_PATH=$B/vpw32/libgcolor.so" "GC_LIB_PATH=$B/vpw16/libgcolor.so" -
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_LIB_PATH=$B/vpw32/libgcolor.so" "GC_LIB_PATH=$B/vpw16/libgcolor.so"
STEPS=10 bash tools/gpu_ab.sh $T uniform10M - "GC_LIB_PATH=$B/vpw32/libgcolor.so" "GC_LIB_PATH=$B/vpw16/libgcolor.so"
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - "GC_LIB_PATH=$B/vpw32/libgcolor.so" "GC_LIB_PATH=$B/vpw16/libgcolor.so"
