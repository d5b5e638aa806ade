set -euo pipefail
# sharded engine rehearsal (P shards on one GPU) and the host protocol's profile
T=r02v5; mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/shard_timing.py rmat24 1 2 4 > gpurun_out/$T/shard_rmat24.txt 2>&1; tail -4 gpurun_out/$T/shard_rmat24.txt | cut -c1-300
timeout -k 10 300 python -u tools/shard_timing.py mesh256 1 2 > gpurun_out/$T/shard_mesh256.txt 2>&1; tail -3 gpurun_out/$T/shard_mesh256.txt | cut -c1-300
timeout -k 10 200 python -u tools/shard_cprof.py rmat24 > gpurun_out/$T/cprof_rmat24.txt 2>&1; head -40 gpurun_out/$T/cprof_rmat24.txt
