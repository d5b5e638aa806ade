"""Shared test helpers.

`-m "not gpu"` tests run in the build container (no GPU); `-m gpu` tests run on an
MI355X through gpurun and always exercise the HIP path through the C-ABI.
"""
import glob
import gzip
import json
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "distributed-graph-coloring-with-pyspark_amd")
GOLDEN = os.path.join(REPO, "tests", "golden", "cases")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)
# the tests share the device with torch's own allocations (resident CSRs, shard buffers): the
# library parks at most 144 GB between calls (half of an MI355X's HBM; the library's default is
# 64 GB, bench.py's one-process-per-GPU runs all but 48 GB)
os.environ.setdefault("GC_ALLOC_IDLE_CAP_GB", "144")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "gpu_staged: GPU test of an opt-in path not yet validated on the GPU "
                                       "(run with -m gpu_staged; promoted to gpu once green)")


def free_port():
    """A TCP port on 127.0.0.1 that was free a moment ago (the OS picks it): rendezvous ports
    for the multi-process tests, instead of random ones that parallel workers can share."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def golden_names():
    return sorted(os.path.basename(p)[: -len(".json.gz")] for p in glob.glob(os.path.join(GOLDEN, "*.json.gz")))


_cache = {}


def load_golden(name):
    if name not in _cache:
        with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as f:
            _cache[name] = json.load(f)
    return _cache[name]


def fixture_csr(rec):
    """(ids, adjacency-by-position, rp, col) exactly as graph.py:15-28 links them
    (a neighbour id resolves to the LAST node carrying that id)."""
    graph = rec["graph"]
    ids = [g[0] for g in graph]
    pos = {}
    for i, vid in enumerate(ids):
        pos[vid] = i
    adj = [[pos[u] for u in g[1]] for g in graph]
    rp = np.zeros(len(adj) + 1, np.int64)
    rp[1:] = np.cumsum([len(a) for a in adj])
    col = np.array([u for a in adj for u in a], dtype=np.int32)
    return ids, adj, rp, col


@pytest.fixture(autouse=True, scope="module")
def _release_device_cache():
    """After each test module, the library's parked device blocks go back to the runtime (the
    allocator keeps up to GC_ALLOC_IDLE_CAP_GB for the next graph of the same size; the next module may
    need that memory for torch tensors).  Only if the module loaded the library."""
    yield
    mod = sys.modules.get("gcolor_amd._native")
    if mod is not None and getattr(mod, "_lib", None) is not None:
        mod._lib.gc_release_cache()


@pytest.fixture(scope="session")
def golden():
    return load_golden
