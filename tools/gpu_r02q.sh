set -euo pipefail
mkdir -p gpurun_out/r02q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02q/pytest.log 2>&1 || { tail -40 gpurun_out/r02q/pytest.log; exit 1; }
tail -2 gpurun_out/r02q/pytest.log
STEPS=3 bash tools/gpu_ab.sh r02q mesh512 - "GC_TICKET_CLOSE=0"
STEPS=3 bash tools/gpu_ab.sh r02q rmat24 -
STEPS=5 bash tools/gpu_ab.sh r02q uniform10M - "GC_TICKET_CLOSE=0"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r02q/mesh512_trace; mkdir -p $OUT; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT" -o run -- python "$ROOT/bench.py" --workload mesh512 --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > "$OUT/trace.log" 2>&1
cd $ROOT; python tools/kstats.py $OUT/run_kernel_stats.csv 5; python tools/gaps.py $OUT/run_kernel_trace.csv 4
