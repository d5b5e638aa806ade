set -euo pipefail
# kernel stats of the seeded R-MAT-24 colouring with pushed pending lists
T=r02v28; mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload rmat24 --priority-seed 1 --steps 1 --warmup 0 --no-cpu-baseline --no-event-timing > $GRAFT_REPO_ROOT/gpurun_out/$T/trace.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/$T/trace.log; exit 1; }
head -14 $GRAFT_REPO_ROOT/gpurun_out/$T/trace/run_kernel_stats.csv | cut -d, -f1-4
rm -f $GRAFT_REPO_ROOT/gpurun_out/$T/trace/run_kernel_trace.csv
