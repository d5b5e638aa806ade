set -euo pipefail
mkdir -p gpurun_out/r02zg
STEPS=3 bash tools/gpu_ab.sh r02zg rmat24 - "GC_GRID_PB=256" "GC_GRID_PB=512" "GC_GRID_CB=256" "GC_GRID_CB=512" "GC_GRID_PB=256 GC_GRID_CB=256" "GC_GRID_R=512" "GC_GRID_R=384" -
STEPS=2 bash tools/gpu_ab.sh r02zg rmat26 - "GC_GRID_PB=256 GC_GRID_CB=256" "GC_GRID_R=512" -
