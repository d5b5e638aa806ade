#!/bin/bash
# Kernel traces (per-launch CSV + stats) of one colouring per workload:
#   bash tools/gpu_trace_wl.sh TAG WORKLOAD [WORKLOAD ...]
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for WL in "$@"; do
  OUT=$ROOT/gpurun_out/$TAG/$WL
  mkdir -p "$OUT"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
    python "$ROOT/bench.py" --workload $WL --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing \
    --json-out "$OUT/bench.json" > "$OUT/trace.log" 2>&1
  cd "$ROOT"
  python tools/round_view.py "$OUT/trace/run_kernel_trace.csv" > "$OUT/round_view.txt"
  head -12 "$OUT/trace/run_kernel_stats.csv"
  cat "$OUT/round_view.txt"
done
