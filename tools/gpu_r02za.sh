set -euo pipefail
mkdir -p gpurun_out/r02za
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02za/pytest.log 2>&1 || { tail -30 gpurun_out/r02za/pytest.log; exit 1; }
tail -2 gpurun_out/r02za/pytest.log
for wl in rmat24 mesh512 rmat26; do
 for m in "--priority-seed 1" "--speculative" "--speculative --priority-seed 1"; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline $m > gpurun_out/r02za/run.log 2>&1 || { tail -5 gpurun_out/r02za/run.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/r02za/run.log').read().strip().splitlines()[-1]);print('$wl [$m]', round(d['ms_per_step'],1),'ms', d['config']['rounds'],'rounds', d['colors_used'],'colours', round(d['value']/1e9,3),'GTEPS', flush=True)" | tee -a gpurun_out/r02za/modes.txt
 done
done
