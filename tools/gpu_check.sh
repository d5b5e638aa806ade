# GPU parity suite + the bench workloads (TAG, then workloads; default: c2 rmat26 mesh512)
set -euo pipefail
TAG=${1:-chk}; shift || true
WLS=${*:-"c2 rmat24 rmat26 mesh512"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for w in $WLS; do
  if [ $w = c2 ]; then a=""; else a="--workload $w"; fi
  timeout -k 10 280 python -u bench.py $a --steps 3 --warmup 1 --no-cpu-baseline --json-out $OUT/bench_$w.json > $OUT/bench_$w.log 2>&1
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));print('$w',round(d['ms_per_step'],2),'ms',round(d['value']/1e9,3),'GTEPS')"
done
