"""gcolor_amd -- MI355X-native graph colouring, a drop-in for the reference's coloring.py.

Hot path: libgcolor.so (HIP/gfx950 kernels behind the C-ABI in include/gcolor.h).
Host side: JSON/CSR I/O, generators, the coloring.py-compatible CLI and the in-process
mirror of graph_coloring / validate_graph_coloring.
"""
from . import _native  # noqa: F401
from .graphio import load_graph_json, write_coloring_json, write_graph_json, csr_from_adjacency  # noqa: F401
from .generators import reference_graph, reference_csr  # noqa: F401

__all__ = ["DeviceGraph", "graph_coloring", "validate_graph_coloring", "load_graph_json",
           "write_coloring_json", "write_graph_json", "reference_graph", "reference_csr"]


def __getattr__(name):
    # GPU-backed names load libgcolor.so lazily (importing the package never needs a GPU)
    if name in ("DeviceGraph", "uniform_csr", "device_count"):
        from . import engine
        return getattr(engine, name)
    if name in ("graph_coloring", "validate_graph_coloring"):
        from . import api
        return getattr(api, name)
    raise AttributeError(name)
