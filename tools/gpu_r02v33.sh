set -euo pipefail
# seeded R-MAT-24 knob pass
T=r02v33; OUT=gpurun_out/$T; mkdir -p $OUT
i=0
for E in "" "GC_GRID_PB=2048" "GC_GRID_C=2048" "GC_GRID_CB=2048" "GC_GRID_RH=8192" "GC_GRID_SH=2048" "GC_BIGROW=1024" "GC_SWEEP_PAD=1" "GC_SWEEP_PAD=4"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -20 $OUT/s$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$i.json'));print('seeded rmat24 [$E]', round(d['ms_per_step'],1),'ms')"
done
