set -euo pipefail
T=r02v34; mkdir -p gpurun_out/$T
export GC_BENCH_BACKEND=gloo GC_BENCH_DEVICE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --steps 2 --warmup 1 --workload uniform1M --json-out gpurun_out/$T/u2.json > gpurun_out/$T/u2.log 2>&1 || { tail -30 gpurun_out/$T/u2.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$T/u2.json'));print(d['ms_per_step'], d['config']['single_gpu_ms'], d['config']['speedup_vs_single_gpu'], d['config']['parallelism'])"
