set -euo pipefail
# C5's graph on one GPU: R-MAT-28 (~8.5e9 adjacency entries)
T=r02v16; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u tools/big_rmat_check.py 28 > gpurun_out/$T/rmat28.log 2>&1 || { tail -30 gpurun_out/$T/rmat28.log; exit 1; }
cat gpurun_out/$T/rmat28.log
