set -euo pipefail
# fused propose + first sweep seam, deferred finish for every shard: GPU shard tests + rehearsal
T=r02v18; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 400 python -u tools/shard_timing.py rmat24 1 2 > gpurun_out/$T/shard_rmat24.txt 2>&1 || { tail -20 gpurun_out/$T/shard_rmat24.txt; exit 1; }
tail -3 gpurun_out/$T/shard_rmat24.txt | cut -c1-200
timeout -k 10 300 python -u tools/shard_timing.py mesh256 1 2 > gpurun_out/$T/shard_mesh256.txt 2>&1 || { tail -20 gpurun_out/$T/shard_mesh256.txt; exit 1; }
tail -3 gpurun_out/$T/shard_mesh256.txt | cut -c1-200
