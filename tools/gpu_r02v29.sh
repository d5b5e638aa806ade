set -euo pipefail
# seeded R-MAT-24 under the new grid / bigrow defaults vs the old ones
T=r02v29; OUT=gpurun_out/$T; mkdir -p $OUT
i=0
for E in "" "GC_GRID_S=384" "GC_GRID_S=384 GC_GRID_PS=1024" "GC_BIGROW=4096" "GC_GRID_S=1024"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -20 $OUT/s$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$i.json'));print('seeded rmat24 [$E]', round(d['ms_per_step'],1),'ms')"
done
