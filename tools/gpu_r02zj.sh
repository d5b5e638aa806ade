set -euo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r02zj; mkdir -p $OUT; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d "$OUT/trace" -o run -- python "$ROOT/bench.py" --workload rmat24 --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > "$OUT/trace.log" 2>&1
cd $ROOT; python tools/round_kernels.py $OUT/trace/run_kernel_trace.csv | tee $OUT/round_kernels.txt
rm -f $OUT/trace/run_kernel_trace.csv
