set -euo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r02zb; mkdir -p $OUT; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python "$ROOT/bench.py" --workload rmat24 --priority-seed 1 --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > "$OUT/trace.log" 2>&1
cd $ROOT; python tools/kstats.py $OUT/trace/run_kernel_stats.csv 16; python tools/sweep_view.py $OUT/trace/run_kernel_trace.csv | head -8; python tools/gaps.py $OUT/trace/run_kernel_trace.csv 4
rm -f $OUT/trace/run_kernel_trace.csv
