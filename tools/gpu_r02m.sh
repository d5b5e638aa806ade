set -euo pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02m/pytest.log 2>&1 || { tail -40 gpurun_out/r02m/pytest.log; exit 1; }
tail -3 gpurun_out/r02m/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02m/smoke.log 2>&1
tail -2 gpurun_out/r02m/smoke.log
bash tools/gpu_profile.sh r02m rmat24
