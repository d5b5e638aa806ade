set -euo pipefail
# round-2 re-entry check: every GPU test, then the default bench line
T=r02v2
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
timeout -k 10 400 python -u bench.py --json-out gpurun_out/$T/bench.json > gpurun_out/$T/bench.log 2>&1 || { tail -30 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log | cut -c1-600
