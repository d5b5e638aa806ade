set -euo pipefail
mkdir -p gpurun_out/r02zl
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02zl/pytest.log 2>&1 || { tail -30 gpurun_out/r02zl/pytest.log; exit 1; }
tail -3 gpurun_out/r02zl/pytest.log
