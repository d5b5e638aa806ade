set -euo pipefail
T=r02v17; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/$T/pytest.log | tail -10
