# grid-size sweep of the round kernels: bash tools/gpu_grid.sh WORKLOAD "P/R/C ..."
set -euo pipefail
WL=$1; shift
mkdir -p gpurun_out/grid
for cfg in $@; do
  IFS=/ read P R C <<< "$cfg"
  GC_GRID_P=$P GC_GRID_R=$R GC_GRID_C=$C timeout -k 10 200 python -u bench.py --workload $WL --steps 4 --warmup 1 --no-cpu-baseline --no-event-timing --json-out gpurun_out/grid/b.json > gpurun_out/grid/b.log 2>&1
  python -c "
import json;d=json.load(open('gpurun_out/grid/b.json')); print('$WL $cfg', round(d['ms_per_step'],2))"
done
