set -euo pipefail
mkdir -p gpurun_out/r02i
STEPS=3 bash tools/gpu_ab.sh r02i mesh512 - "GC_GRID_P=512 GC_GRID_R=512 GC_GRID_C=512" "GC_GRID_P=256 GC_GRID_R=256 GC_GRID_C=256" "GC_BATCH_MAX=16" "GC_GRID_P=2048 GC_GRID_R=2048 GC_GRID_C=2048"
bash tools/gpu_trace_ab.sh r02i mesh512 -
