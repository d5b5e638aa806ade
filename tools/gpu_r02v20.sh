set -euo pipefail
# A/B: GC_BIGROW (winners with longer in-rows go to the grid-wide k_commit_big)
T=r02v20; mkdir -p gpurun_out/$T
STEPS=5 bash tools/gpu_ab.sh $T rmat24 - "GC_BIGROW=512" "GC_BIGROW=1024" "GC_BIGROW=2048" "GC_BIGROW=8192" - "GC_BIGROW=1024"
STEPS=3 bash tools/gpu_ab.sh $T rmat26 - "GC_BIGROW=1024" "GC_BIGROW=2048"
