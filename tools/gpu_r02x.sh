set -euo pipefail
mkdir -p gpurun_out/r02x
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant_b.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02x/pytest_b.log 2>&1 || { tail -30 gpurun_out/r02x/pytest_b.log; exit 1; }
tail -2 gpurun_out/r02x/pytest_b.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02x/pytest.log 2>&1 || { tail -30 gpurun_out/r02x/pytest.log; exit 1; }
tail -2 gpurun_out/r02x/pytest.log
timeout -k 10 300 python -u bench.py --workload uniform10M --variant B --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02x/b_uni.log 2>&1
tail -1 gpurun_out/r02x/b_uni.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload rmat24 --variant B --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02x/b_rmat24.log 2>&1
tail -1 gpurun_out/r02x/b_rmat24.log | cut -c1-200
