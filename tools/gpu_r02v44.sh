set -euo pipefail
T=r02v44; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
STEPS=5 bash tools/gpu_ab.sh $T mesh512 - -
STEPS=5 bash tools/gpu_ab.sh $T rmat24 -
