"""Drop-in for the reference's coloring_optimized.py (variant B semantics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gcolor_amd.cli import main  # noqa: E402


def graph_coloring(graph_rdd, numOfColors, sc=None):
    from gcolor_amd.api import graph_coloring as _gc
    return _gc(graph_rdd, numOfColors, sc, variant="B")


def validate_graph_coloring(graph_rdd):
    from gcolor_amd.api import validate_graph_coloring as _v
    return _v(graph_rdd)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] + ["--variant", "B"]))
