set -euo pipefail
# variant B fold pass grids (R-MAT-24, C2)
T=r02v36; OUT=gpurun_out/$T; mkdir -p $OUT
i=0
for E in "" "GC_GRID_BA=2048" "GC_GRID_BA=4096" "GC_GRID_BA=512" "GC_GRID_BE=512" "GC_GRID_BE=2048" "GC_GRID_BA=4096 GC_GRID_BE=512"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --variant B --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$i.json'));print('B rmat24 [$E]', round(d['ms_per_step'],1),'ms')"
done
for E in "" "GC_GRID_BA=4096"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload uniform10M --variant B --steps 5 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$i.json'));print('B C2 [$E]', round(d['ms_per_step'],2),'ms')"
done
