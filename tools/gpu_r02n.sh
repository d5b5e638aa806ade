set -euo pipefail
ROOT=$(pwd); export TMPDIR=/tmp
i=0
for E in "-" "GC_GRID_C=256" "GC_GRID_C=512" "GC_GRID_C=2048" "GC_GRID_P=256 GC_GRID_R=256" "GC_GRID_P=2048 GC_GRID_R=2048"; do
  i=$((i+1)); [ "$E" = "-" ] && E=""
  OUT=$ROOT/gpurun_out/r02n/mesh512_t$i; mkdir -p "$OUT"
  for kv in $E; do export "$kv"; done
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
    python "$ROOT/bench.py" --workload mesh512 --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > "$OUT/trace.log" 2>&1
  cd "$ROOT"
  for kv in $E; do unset "${kv%%=*}"; done
  echo "== [$E]"; python tools/kstats.py "$OUT/trace/run_kernel_stats.csv" 6
done
