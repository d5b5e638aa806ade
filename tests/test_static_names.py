"""Every Python file of the repository reads only names it defines or imports
(tools/undefined_names.py) -- in particular the staged GPU tests and GPU-only tools, which no
CPU run executes."""
import glob
import os
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import undefined_names  # noqa: E402


def _files():
    pats = ["*.py", "tests/*.py", "tools/*.py", "oracle/*.py", "distributed-graph-coloring-with-pyspark_amd/*.py",
            "distributed-graph-coloring-with-pyspark_amd/gcolor_amd/*.py", "tests/golden/*.py"]
    return sorted({p for pat in pats for p in glob.glob(os.path.join(REPO, pat))})


def test_no_undefined_names():
    files = _files()
    assert len(files) > 40
    bad = [(os.path.relpath(p, REPO), *x) for p in files for x in undefined_names.check(p)]
    assert not bad, bad
