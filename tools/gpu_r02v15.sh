set -euo pipefail
# adjacency beyond 2^31 entries: R-MAT-27 engine + validate + one shard
T=r02v15; mkdir -p gpurun_out/$T
timeout -k 10 900 python -u tools/big_rmat_check.py 27 shard > gpurun_out/$T/rmat27.log 2>&1 || { tail -30 gpurun_out/$T/rmat27.log; exit 1; }
cat gpurun_out/$T/rmat27.log
