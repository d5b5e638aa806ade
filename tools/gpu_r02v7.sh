set -euo pipefail
# deferred shard finish / async hub JP (per-rank halts): GPU shard tests, rehearsal timing, kernel trace of P=1
T=r02v7; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 400 python -u tools/shard_timing.py rmat24 1 2 4 > gpurun_out/$T/shard_rmat24.txt 2>&1 || { tail -20 gpurun_out/$T/shard_rmat24.txt; exit 1; }
tail -4 gpurun_out/$T/shard_rmat24.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o shard -- python3 $GRAFT_REPO_ROOT/tools/shard_cprof.py rmat24 > $GRAFT_REPO_ROOT/gpurun_out/$T/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/$T/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1 | xargs head -25 | cut -d, -f1-4
