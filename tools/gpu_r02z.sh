set -euo pipefail
mkdir -p gpurun_out/r02z
for wl in rmat24 mesh512 uniform10M rmat26; do
 for m in "" "--priority-seed 1" "--speculative" "--speculative --priority-seed 1"; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline $m > gpurun_out/r02z/run.log 2>&1 || { tail -5 gpurun_out/r02z/run.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/r02z/run.log').read().strip().splitlines()[-1]);print('$wl [$m]', round(d['ms_per_step'],1),'ms', d['config']['rounds'],'rounds', d['colors_used'],'colours', round(d['value']/1e9,3),'GTEPS')"
 done
done
