#!/bin/bash
# One GPU session on the MI355X box (run through gpurun from the repo root):
#   1. the GPU parity suite, 2. the default bench line, 3. rocprofv3 kernel-trace stats of
#   the same bench command, 4./5. FETCH_SIZE and WRITE_SIZE PMC passes (separate runs,
#   counters only -- never combined with other tracing).
# Every GPU step has its own time limit and the steps are chained: the first failure ends
# the script.  Output lands in gpurun_out/ (merged back by gpurun).
# Usage: bash tools/gpu_profile.sh [TAG] [extra bench args...]
set -euo pipefail
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u bench.py --json-out "$OUT/bench.json" "$@" > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
  python "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/pmc_fetch" -o run -- \
  python "$ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 0 "$@" > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$OUT/pmc_write" -o run -- \
  python "$ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 0 "$@" > "$OUT/pmc_write.log" 2>&1
echo "gpu_profile done: $OUT"
