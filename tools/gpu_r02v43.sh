set -euo pipefail
# commit grid sweep (mesh, R-MAT-24, C2)
T=r02v43; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - "GC_GRID_C=512" "GC_GRID_C=640" "GC_GRID_C=768" "GC_GRID_C=896" -
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_GRID_C=640" "GC_GRID_C=768" -
STEPS=10 bash tools/gpu_ab.sh $T uniform10M - "GC_GRID_C=640" "GC_GRID_C=768"
