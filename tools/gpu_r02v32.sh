set -euo pipefail
# larger JP grids only where heavy vertices take workgroups (heavy_wg)
T=r02v32; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload rmat24 --priority-seed 1 --steps 3 --warmup 1 --no-cpu-baseline --no-event-timing --json-out $OUT/seeded.json > $OUT/seeded.log 2>&1 || { tail -20 $OUT/seeded.log; exit 1; }
python -c "import json;d=json.load(open('$OUT/seeded.json'));print('seeded rmat24', round(d['ms_per_step'],1),'ms')"
STEPS=3 bash tools/gpu_ab.sh $T rmat24 - "GC_HUB_T=off"
STEPS=5 bash tools/gpu_ab.sh $T mesh512 -
STEPS=10 bash tools/gpu_ab.sh $T uniform10M -
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
