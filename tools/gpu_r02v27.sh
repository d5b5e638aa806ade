set -euo pipefail
# seeded ranks with pushed pending lists: priority parity, then the seeded bench A/B
T=r02v27; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_priority.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
OUT=gpurun_out/$T; 
for E in "" "GC_HPUSH=0" "GC_HPUSH=2"; do
  timeout -k 10 300 env $E python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --json-out $OUT/seeded_${E:-default}.json > $OUT/seeded_${E:-default}.log 2>&1 || { tail -20 $OUT/seeded_${E:-default}.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/seeded_${E:-default}.json'));print('seeded rmat24 [$E]', round(d['ms_per_step'],1),'ms', d['config']['rounds'],'rounds', d['colors_used'],'colours')"
done
