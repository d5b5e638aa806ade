set -euo pipefail
# sweep grid by mode: hub JP 256 (GC_GRID_S), workgroup-per-heavy 1024 (GC_GRID_SH)
T=r02v30; OUT=gpurun_out/$T; mkdir -p $OUT
i=0
for E in "" "GC_GRID_SH=2048" "GC_GRID_SH=1536"; do
  i=$((i+1))
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -20 $OUT/s$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$i.json'));print('seeded rmat24 [$E]', round(d['ms_per_step'],1),'ms')"
done
STEPS=3 bash tools/gpu_ab.sh $T rmat24 - "GC_HUB_T=off" "GC_HUB_T=off GC_GRID_SH=384"
STEPS=5 bash tools/gpu_ab.sh $T mesh512 -
STEPS=10 bash tools/gpu_ab.sh $T uniform10M -
timeout -k 10 600 python -u -m pytest tests/test_gpu_priority.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
