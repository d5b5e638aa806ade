set -euo pipefail
mkdir -p gpurun_out/hubs
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hubs/pytest_hubs.log 2>&1 || { tail -60 gpurun_out/hubs/pytest_hubs.log; exit 1; }
tail -3 gpurun_out/hubs/pytest_hubs.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hubs/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/hubs/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/hubs/pytest_gpu.log
for w in rmat24 uniform10M; do
  timeout -k 10 280 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --json-out gpurun_out/hubs/bench_$w.json > gpurun_out/hubs/bench_$w.log 2>&1
  tail -1 gpurun_out/hubs/bench_$w.log | cut -c1-300
done
