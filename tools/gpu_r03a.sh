set -uo pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "partition or rows_list or rejects or golden_graphs or repeat" > $O/t1.log 2>&1 || { tail -60 $O/t1.log; exit 1; }
tail -3 $O/t1.log
timeout -k 10 300 python -u tools/step_timing.py rmat24 4 > $O/step24.log 2>&1 || { tail -30 $O/step24.log; exit 1; }
cat $O/step24.log
