set -euo pipefail
# atomic-free shard in-CSR for symmetric graphs: shard tests + set-up time
T=r02v11; mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
timeout -k 10 300 python -u - > gpurun_out/$T/setup.txt 2>&1 <<'PY'
import sys, time
sys.path.insert(0, "distributed-graph-coloring-with-pyspark_amd")
import torch
from gcolor_amd import shard as sh
from gcolor_amd.engine import DeviceGraph
torch.cuda.set_device(0)
dg = DeviceGraph.rmat(24, 16, seed=1)
rp, _ = dg.export(col=False)
for P in (1, 8):
    lo, hi = sh.balanced_ranges(rp, P)[0]
    t = time.time(); s = sh.HipShard(dg, lo, hi); torch.cuda.synchronize(); print(f"P={P} shard 0 create {time.time() - t:.3f} s", flush=True); s.close()
PY
cat gpurun_out/$T/setup.txt
timeout -k 10 300 python -u tools/shard_timing.py rmat24 1 > gpurun_out/$T/shard_rmat24.txt 2>&1; tail -2 gpurun_out/$T/shard_rmat24.txt | cut -c1-200
