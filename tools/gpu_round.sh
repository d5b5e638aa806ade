set -euo pipefail
TAG=${1:-r01}
bash tools/gpu_profile.sh $TAG
mkdir -p gpurun_out/$TAG/wl
for w in rmat24 rmat26 mesh512 mesh256; do
  timeout -k 10 280 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --json-out gpurun_out/$TAG/wl/bench_$w.json > gpurun_out/$TAG/wl/bench_$w.log 2>&1
  tail -1 gpurun_out/$TAG/wl/bench_$w.log | cut -c1-250
done
