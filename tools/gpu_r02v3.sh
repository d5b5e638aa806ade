set -euo pipefail
# tail workgroup of 8/16 waves and larger tail limits: parity under them, then A/B on R-MAT
T=r02v3
mkdir -p gpurun_out/$T
GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096 GC_TAIL_HMAX_HUB=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hubs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest16.log 2>&1 || { tail -30 gpurun_out/$T/pytest16.log; exit 1; }
tail -1 gpurun_out/$T/pytest16.log
STEPS=3 bash tools/gpu_ab.sh $T rmat24 - "GC_TAIL_WAVES=16" "GC_TAIL_WAVES=16 GC_TAIL_LMAX=2048" "GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096" "GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096 GC_TAIL_HMAX_HUB=512" "GC_TAIL_WAVES=8 GC_TAIL_LMAX=2048" -
STEPS=2 bash tools/gpu_ab.sh $T rmat26 - "GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096" "GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096 GC_TAIL_HMAX_HUB=512" -
STEPS=5 bash tools/gpu_ab.sh $T uniform10M - "GC_TAIL_WAVES=16 GC_TAIL_LMAX=4096" -
