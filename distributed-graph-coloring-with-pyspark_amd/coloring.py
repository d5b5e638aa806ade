"""Drop-in for the reference's coloring.py: same CLI, stdout and JSON files; the
colouring runs on an MI355X through libgcolor.so.

    python coloring.py --input graph.json --output-coloring colors.json
    python coloring.py --node-count 10000 --max-degree 8 --output-coloring colors.json

In-process: graph_coloring(nodes, k) / validate_graph_coloring(nodes) mirror
coloring.py:73 and :149.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gcolor_amd.cli import main  # noqa: E402


def graph_coloring(graph_rdd, numOfColors, sc=None):
    from gcolor_amd.api import graph_coloring as _gc
    return _gc(graph_rdd, numOfColors, sc, variant="A")


def validate_graph_coloring(graph_rdd):
    from gcolor_amd.api import validate_graph_coloring as _v
    return _v(graph_rdd)


if __name__ == "__main__":
    sys.exit(main())
