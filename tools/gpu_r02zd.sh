set -euo pipefail
mkdir -p gpurun_out/r02zd
STEPS=3 bash tools/gpu_ab.sh r02zd rmat24 - "GC_GRID_R=512" "GC_GRID_R=768" "GC_GRID_P=512 GC_GRID_C=512" "GC_TAIL_HMAX_HUB=256" "GC_BATCH_MAX=8" -
STEPS=2 bash tools/gpu_ab.sh r02zd rmat26 - "GC_GRID_R=512" "GC_TAIL_HMAX_HUB=256" "GC_BATCH_MAX=8" -
