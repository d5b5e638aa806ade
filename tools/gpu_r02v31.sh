set -euo pipefail
# seeded R-MAT-24: first-sweep (k_resolve) grid
T=r02v31; OUT=gpurun_out/$T; mkdir -p $OUT
i=0
for E in "" "GC_GRID_R=2048" "GC_GRID_R=4096" "GC_GRID_SH=2048 GC_GRID_R=2048"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -20 $OUT/s$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$i.json'));print('seeded rmat24 [$E]', round(d['ms_per_step'],1),'ms')"
done
STEPS=3 bash tools/gpu_ab.sh $T rmat24 - "GC_GRID_R=2048"
