set -euo pipefail
# knob pass 3 on the current defaults (R-MAT-24)
T=r02v25; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_GRID_PB=256" "GC_GRID_PB=512" "GC_GRID_PS=256" "GC_GRID_PS=384" "GC_GRID_S=192" "GC_HUB_T=256" "GC_TAIL_HMAX_HUB=192" "GC_BIGROW=1024" "GC_BIGROW=3072" "GC_GRID_CB=512" "GC_GRID_C=768" -
