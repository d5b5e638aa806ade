set -euo pipefail
# bench.py's multi-rank path end to end on one GPU (2 ranks over gloo), weak and strong
T=r02v19; mkdir -p gpurun_out/$T
export GC_BENCH_BACKEND=gloo GC_BENCH_DEVICE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --json-out gpurun_out/$T/weak2.json > gpurun_out/$T/weak2.log 2>&1 || { tail -30 gpurun_out/$T/weak2.log; exit 1; }
tail -1 gpurun_out/$T/weak2.log | cut -c1-700
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 2 --warmup 1 --workload mesh256 --scaling strong --json-out gpurun_out/$T/mesh2.json > gpurun_out/$T/mesh2.log 2>&1 || { tail -30 gpurun_out/$T/mesh2.log; exit 1; }
tail -1 gpurun_out/$T/mesh2.log | cut -c1-500
