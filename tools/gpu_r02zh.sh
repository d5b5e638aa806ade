set -euo pipefail
mkdir -p gpurun_out/r02zh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zh/pytest.log 2>&1 || { tail -30 gpurun_out/r02zh/pytest.log; exit 1; }
tail -2 gpurun_out/r02zh/pytest.log
for m in "--priority-seed 1" "--speculative --priority-seed 1"; do
  timeout -k 10 300 python -u bench.py --workload rmat24 --steps 3 --warmup 1 --no-cpu-baseline $m > gpurun_out/r02zh/run.log 2>&1 || { tail -5 gpurun_out/r02zh/run.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r02zh/run.log').read().strip().splitlines()[-1]);print('rmat24 [$m]', round(d['ms_per_step'],1),'ms', d['config']['rounds'],'rounds', d['colors_used'],'colours', flush=True)"
done
STEPS=2 bash tools/gpu_ab.sh r02zh rmat24 "GC_HUB_T=off"
timeout -k 10 400 python -u tools/shard_timing.py rmat24 1 2 > gpurun_out/r02zh/shard.log 2>&1 || { tail -5 gpurun_out/r02zh/shard.log; exit 1; }
cat gpurun_out/r02zh/shard.log
