set -euo pipefail
mkdir -p gpurun_out/r02zi
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02zi/pytest_shard.log 2>&1 || { tail -30 gpurun_out/r02zi/pytest_shard.log; exit 1; }
tail -2 gpurun_out/r02zi/pytest_shard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zi/pytest.log 2>&1 || { tail -30 gpurun_out/r02zi/pytest.log; exit 1; }
tail -2 gpurun_out/r02zi/pytest.log
timeout -k 10 400 python -u tools/shard_timing.py rmat24 1 2 > gpurun_out/r02zi/shard.log 2>&1 || { tail -5 gpurun_out/r02zi/shard.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02zi/shard.log | tail -3
