#!/bin/bash
# Kernel traces of one colouring under several environments:
#   bash tools/gpu_trace_ab.sh TAG WORKLOAD "ENV1" "ENV2" ...   ("-" = defaults)
set -euo pipefail
TAG=$1; WL=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E=""
  OUT=$ROOT/gpurun_out/$TAG/${WL}_t$i
  mkdir -p "$OUT"
  for kv in $E; do export "$kv"; done
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
    python "$ROOT/bench.py" --workload $WL --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > "$OUT/trace.log" 2>&1
  cd "$ROOT"
  for kv in $E; do unset "${kv%%=*}"; done
  echo "== $WL [$E]"
  python tools/sweep_view.py "$OUT/trace/run_kernel_trace.csv" | tee "$OUT/sweep_view.txt"
done
