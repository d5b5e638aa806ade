set -euo pipefail
# speculative mode: heavy proposers a workgroup each with early exit
T=r02v38; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_priority.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for A in "--speculative" "--speculative --priority-seed 1"; do
  for W in rmat24 mesh512; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --workload $W $A --steps 2 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -20 $OUT/s$i.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/s$i.json'));print('$W [$A]', round(d['ms_per_step'],1),'ms', d['config']['rounds'], d['colors_used'])"
  done
done
