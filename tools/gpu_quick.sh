set -euo pipefail
mkdir -p gpurun_out/r01b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01b/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r01b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r01b/pytest_gpu.log
timeout -k 10 300 python -u bench.py --json-out gpurun_out/r01b/bench.json > gpurun_out/r01b/bench.log 2>&1
tail -1 gpurun_out/r01b/bench.log
