# rocprofv3 kernel-trace stats of one bench workload: bash tools/gpu_prof_wl.sh TAG WORKLOAD
set -euo pipefail
TAG=$1; WL=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u "$ROOT/bench.py" --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-200
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
  python "$ROOT/bench.py" --workload $WL --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/trace.log" 2>&1
head -25 "$OUT/trace/run_kernel_stats.csv"
