set -euo pipefail
mkdir -p gpurun_out/r02s
B=$(pwd)/build_variants
for wl in mesh512 rmat24; do
STEPS=3 bash tools/gpu_ab.sh r02s $wl - "GC_LIB_PATH=$B/old/libgcolor.so" "GC_LIB_PATH=$B/cs1/libgcolor.so" "GC_LIB_PATH=$B/fs2/libgcolor.so" "GC_LIB_PATH=$B/nopf/libgcolor.so" "GC_CLAIM_DIRECT=1" -
done
