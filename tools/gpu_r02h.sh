set -euo pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02h/pytest.log 2>&1 || { tail -40 gpurun_out/r02h/pytest.log; exit 1; }
tail -3 gpurun_out/r02h/pytest.log
timeout -k 10 300 python -u tools/shard_timing.py mesh256 1 2 4 8 > gpurun_out/r02h/shard_mesh256.log 2>&1
tail -1 gpurun_out/r02h/shard_mesh256.log
timeout -k 10 300 python -u tools/shard_timing.py uniform10M 1 2 4 8 > gpurun_out/r02h/shard_uniform10M.log 2>&1
tail -1 gpurun_out/r02h/shard_uniform10M.log
