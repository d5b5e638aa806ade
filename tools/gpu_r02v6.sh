set -euo pipefail
# deferred shard finish / async hub JP: GPU shard tests, engine parity, rehearsal timing
T=r02v6; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 300 python -u tools/shard_timing.py rmat24 1 2 4 > gpurun_out/$T/shard_rmat24.txt 2>&1; tail -4 gpurun_out/$T/shard_rmat24.txt | cut -c1-200
timeout -k 10 200 python -u tools/shard_cprof.py rmat24 > gpurun_out/$T/cprof_rmat24.txt 2>&1; head -30 gpurun_out/$T/cprof_rmat24.txt
