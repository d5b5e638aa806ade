#!/bin/bash
# A/B bench runs: bash tools/gpu_ab.sh TAG WORKLOAD "ENV1" "ENV2" ...  (each ENV a space-separated
# list of VAR=value, or "-" for the defaults); bench lines in gpurun_out/TAG/
set -euo pipefail
TAG=$1; WL=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E=""
  timeout -k 10 300 env $E python -u bench.py --workload $WL --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --json-out $OUT/${WL}_$i.json > $OUT/${WL}_$i.log 2>&1
  python -c "import json,sys;d=json.load(open('$OUT/${WL}_$i.json'));r=d['roofline'];print('$WL [$E]', round(d['ms_per_step'],1),'ms', d['config']['rounds'],'rounds', 'dom',r['kernel'], round(r['share_of_step'],3), 'launches',r['launches_per_step'], 'avg_us', round(r['avg_launch_ms']*1e3,1))"
done
