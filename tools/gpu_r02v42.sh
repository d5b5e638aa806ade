set -euo pipefail
# mesh knob pass on the current build
T=r02v42; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - "GC_GRID_C=768" "GC_GRID_C=1536" "GC_GRID_R=512" "GC_GRID_R=768" "GC_GRID_R=1536" "GC_BATCH_MAX=8" "GC_BATCH_MAX=16" "GC_GRID_C=1536 GC_GRID_R=768" -
