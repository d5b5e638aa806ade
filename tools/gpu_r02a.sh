set -euo pipefail
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread --durations=0 > gpurun_out/r02a/fullsize.log 2>&1 || { tail -30 gpurun_out/r02a/fullsize.log; exit 1; }
tail -15 gpurun_out/r02a/fullsize.log
bash tools/gpu_profile.sh r02a rmat24
