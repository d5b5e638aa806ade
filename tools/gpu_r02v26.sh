set -euo pipefail
# per-launch kernel trace of one R-MAT-24 colouring (round structure of the JP sweeps)
bash tools/gpu_trace_wl.sh r02v26 rmat24 > /dev/null 2>&1 || { tail -20 gpurun_out/r02v26/rmat24/trace.log; exit 1; }
gzip -k gpurun_out/r02v26/rmat24/trace/run_kernel_trace.csv
ls -la gpurun_out/r02v26/rmat24/trace/
