set -euo pipefail
# knob re-tune on the current build (R-MAT-24)
T=r02v22; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_HUB_T=256" "GC_HUB_T=384" "GC_HUB_T=768" "GC_BATCH_MAX=8" "GC_BATCH_MAX=16" "GC_SWEEP_PAD=1" "GC_SWEEP_PAD=3" "GC_TAIL_HMAX_HUB=64" "GC_TAIL_HMAX_HUB=256" "GC_GRID_S=256" "GC_GRID_S=512" "GC_GRID_C=512" "GC_GRID_P=512" "GC_GRID_R=512" "GC_GRID_CB=512" -
