#!/bin/bash
# One profiling session of one bench workload on the MI355X box (run through gpurun from
# the repo root):
#   1. the bench line, 2. rocprofv3 kernel-trace stats of the same bench command,
#   3./4. FETCH_SIZE and WRITE_SIZE PMC passes (separate runs, counters only -- never
#   combined with other tracing), 5. the per-kernel summary profiles/pmc/<workload>.json
#   that bench.py reads for `traffic` (copied into the tree; commit it).
# The counter passes run at 3 and at 1 timed steps; the whole step's bytes ("_step") are
# their difference / 2 (setup, warmup and everything else cancel).
# Every GPU step has its own time limit and the steps are chained: the first failure ends
# the script.  Output lands in gpurun_out/<tag>/<workload> (merged back by gpurun).
# Usage: bash tools/gpu_profile.sh TAG WORKLOAD [extra bench args...]
set -euo pipefail
TAG=$1; WL=$2
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
SUF=$(echo "$*" | tr -c 'A-Za-z0-9\n' '_' | sed 's/^_*//; s/_*$//')
OUT=$ROOT/gpurun_out/$TAG/$WL${SUF:+_$SUF}  # one directory per workload and argument set
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python -u bench.py --workload $WL --json-out "$OUT/bench.json" "$@" > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-600
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
  python "$ROOT/bench.py" --workload $WL --no-cpu-baseline --no-north-star --no-variant-b --no-end-to-end --steps 3 --warmup 1 "$@" > "$OUT/trace.log" 2>&1
# counters: the same command at 3 and at 1 timed steps; per-kernel numbers from the first,
# the whole step's bytes from the difference / 2 (setup, warmup and the rest cancel)
for K in 3 1; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/pmc_fetch$K" -o run -- \
    python "$ROOT/bench.py" --workload $WL --no-cpu-baseline --no-north-star --no-variant-b --no-end-to-end --no-event-timing --steps $K --warmup 1 "$@" > "$OUT/pmc_fetch$K.log" 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$OUT/pmc_write$K" -o run -- \
    python "$ROOT/bench.py" --workload $WL --no-cpu-baseline --no-north-star --no-variant-b --no-end-to-end --no-event-timing --steps $K --warmup 1 "$@" > "$OUT/pmc_write$K.log" 2>&1
done
cd "$ROOT"
python tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"
python tools/sweep_view.py "$OUT/trace/run_kernel_trace.csv" > "$OUT/sweep_view.txt" || true
python tools/gaps.py "$OUT/trace/run_kernel_trace.csv" 8 > "$OUT/gaps.txt" || true
# the raw per-dispatch CSVs run to tens of MB per workload (gpurun merges back <= 64 MiB):
# keep the summaries above and the kernel stats only
rm -f "$OUT"/trace/run_kernel_trace.csv "$OUT"/pmc_*/run_counter_collection.csv
echo "gpu_profile done: $OUT"
