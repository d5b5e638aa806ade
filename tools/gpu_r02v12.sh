set -euo pipefail
# A/B: JP sweeps without their diagnostic stats counters
T=r02v12; mkdir -p gpurun_out/$T
B=$(pwd)/build_variants
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_LIB_PATH=$B/nostat/libgcolor.so" - "GC_LIB_PATH=$B/nostat/libgcolor.so"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_LIB_PATH=$B/nostat/libgcolor.so"
