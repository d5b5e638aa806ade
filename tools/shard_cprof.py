"""cProfile of one P=1 sharded colouring (host protocol cost per seam), over a one-rank
RCCL group (argv[2] == "threads": the thread transport)."""
import cProfile, os, pstats, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd"))
import torch
from gcolor_amd import shard as sh
from gcolor_amd.engine import DeviceGraph
torch.cuda.set_device(0)
wl = sys.argv[1] if len(sys.argv) > 1 else "rmat24"
dg = DeviceGraph.rmat(int(wl[4:]), 16, seed=1) if wl.startswith("rmat") else DeviceGraph.mesh(*(3 * [int(wl[4:])]))
rp, _ = dg.export(col=False)
s = sh.HipShard(dg, 0, dg.n)
if len(sys.argv) > 2 and sys.argv[2] == "threads":
    hub = sh.ThreadHub(1)
    comm = sh.ThreadTransport(hub, 0)
else:
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29513", RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    comm = sh.TorchTransport()
sh.shard_color(s, comm, want_colors=False)
pr = cProfile.Profile()
pr.enable()
r = sh.shard_color(s, comm, want_colors=False)
torch.cuda.synchronize()
pr.disable()
print("exchanges", r.exchanges, "rounds", r.rounds)
pstats.Stats(pr).sort_stats("tottime").print_stats(28)
