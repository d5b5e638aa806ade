# SQ / TCC counter passes (separate runs) over one bench step: bash tools/gpu_pmc_sq.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES -T -f csv -d "$OUT/sq" -o run -- \
  python "$ROOT/bench.py" --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv -d "$OUT/tcc" -o run -- \
  python "$ROOT/bench.py" --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$OUT/tcc.log" 2>&1
echo done
