set -euo pipefail
mkdir -p gpurun_out/r02ze
STEPS=3 bash tools/gpu_ab.sh r02ze rmat24 - "GC_GRID_S=512" "GC_GRID_S=384" "GC_GRID_S=256" "GC_GRID_R=512 GC_GRID_S=512" "GC_GRID_S=512 GC_SWEEP_PAD=3" -
STEPS=2 bash tools/gpu_ab.sh r02ze rmat26 - "GC_GRID_S=512" "GC_GRID_S=384" "GC_GRID_S=256" -
STEPS=5 bash tools/gpu_ab.sh r02ze uniform10M - "GC_GRID_S=512" "GC_GRID_S=256"
STEPS=3 bash tools/gpu_ab.sh r02ze mesh512 - "GC_GRID_S=512" "GC_GRID_R=512"
