set -euo pipefail
# variant B: admission grid 2048 when heavy vertices exist; parity and benches
T=r02v37; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant_b.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for W in rmat24 rmat24 uniform10M; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --workload $W --variant B --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$i.json'));print('B $W', round(d['ms_per_step'],2),'ms', d['config']['rounds'], d['colors_used'])"
done
