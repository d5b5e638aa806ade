"""cProfile of one P=1 sharded colouring (host protocol cost per seam)."""
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
hub = sh.ThreadHub(1)
sh.shard_color(s, sh.ThreadTransport(hub, 0), want_colors=False)
pr = cProfile.Profile()
pr.enable()
r = sh.shard_color(s, sh.ThreadTransport(hub, 0), want_colors=False)
torch.cuda.synchronize()
pr.disable()
print("exchanges", r.exchanges, "rounds", r.rounds)
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
