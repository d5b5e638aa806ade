set -euo pipefail
# grid re-tune, second pass (R-MAT-24 / R-MAT-26 / mesh / C2)
T=r02v23; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_GRID_S=256" "GC_GRID_S=192" "GC_GRID_S=128" "GC_GRID_S=256 GC_GRID_P=512" "GC_GRID_S=256 GC_GRID_P=512 GC_GRID_C=512" "GC_GRID_P=256" - "GC_GRID_S=256 GC_GRID_P=512"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_GRID_S=256" "GC_GRID_S=256 GC_GRID_P=512"
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - "GC_GRID_S=256 GC_GRID_P=512"
STEPS=10 bash tools/gpu_ab.sh $T uniform10M - "GC_GRID_S=256 GC_GRID_P=512"
