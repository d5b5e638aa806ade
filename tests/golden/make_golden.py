#!/usr/bin/env python3
"""Generate golden vectors by executing the reference's OWN code (build container only).

TEST INFRASTRUCTURE. This script is the only place that touches ``/root/reference``:
it runs the reference's unmodified ``coloring.py`` (variant A) and
``coloring_optimized.py`` (variant B) through ``runpy`` with the sequential
single-partition stub in ``tests/golden/stub_pyspark`` first on ``sys.path``
(SURVEY.md §8c, Appendix A), and records inputs and outputs as data fixtures under
``tests/golden/cases/``.  Nothing here is imported by the product, and the GPU box
never sees ``/root/reference`` -- only the committed fixtures travel.

Recorded per case and variant:
  * ``cli``  : the reference CLI run (``coloring.py:165-243``): normalised stdout
               transcript, exit status, output colouring (ids + colours in output order)
               and the sha256 of the exact output-file bytes; ``hang`` when the
               reference loops forever (SURVEY Q1 -- detected as the same
               "Uncolored nodes remaining" line repeated ``HANG_REPEATS`` times).
  * ``run``  : ``graph_coloring(rdd, k)`` called directly with an unbounded ``k``
               (``coloring.py:73``): per-round uncoloured counts, final colours in file
               order, and the round in which each vertex became coloured (from the
               per-round ``broadcast_colors`` maps, ``coloring.py:135-137``).

Usage: python tests/golden/make_golden.py [--jobs 6] [--only NAME ...]
"""
import argparse
import builtins
import contextlib
import gzip
import hashlib
import io
import json
import multiprocessing as mp
import os
import random
import re
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
STUB = os.path.join(HERE, "stub_pyspark")
OUT_DIR = os.path.join(HERE, "cases")
HANG_REPEATS = 6
UNBOUNDED_K = 1 << 30

VARIANT_FILE = {"A": "coloring.py", "B": "coloring_optimized.py"}


class _Hang(Exception):
    pass


def _setup_paths():
    for p in (REF, STUB):
        if p in sys.path:
            sys.path.remove(p)
    sys.path.insert(0, REF)
    sys.path.insert(0, STUB)


@contextlib.contextmanager
def _watch_prints(lines):
    """Capture print() output; abort the reference when it spins."""
    real_print = builtins.print
    state = {"last": None, "rep": 0}

    def fake_print(*args, **kwargs):
        buf = io.StringIO()
        kwargs.pop("file", None)
        real_print(*args, file=buf, **kwargs)
        for line in buf.getvalue().splitlines():
            lines.append(line)
            if line.startswith("Uncolored nodes remaining"):
                if line == state["last"]:
                    state["rep"] += 1
                    if state["rep"] >= HANG_REPEATS:
                        raise _Hang()
                else:
                    state["last"], state["rep"] = line, 1
            else:
                state["last"], state["rep"] = None, 0

    builtins.print = fake_print
    try:
        yield
    finally:
        builtins.print = real_print


def _normalise(lines):
    out = []
    for ln in lines:
        ln = re.sub(r"^Iteration time: [0-9.]+ seconds$", "Iteration time: <t> seconds", ln)
        ln = re.sub(r"^Total execution time: [0-9.]+ seconds$", "Total execution time: <t> seconds", ln)
        out.append(ln)
    return out


def _run_cli(variant, argv, seed=None):
    """Run the reference CLI in-process; return the recorded dict."""
    import runpy
    _setup_paths()
    lines = []
    rec = {"argv": argv, "hang": False, "exit": 0}
    with tempfile.TemporaryDirectory() as td:
        out_path = os.path.join(td, "colors.json")
        graph_out = os.path.join(td, "graph_out.json")
        full = ["coloring.py"] + [a.replace("@OUT", out_path).replace("@GRAPH_OUT", graph_out) for a in argv]
        sys.argv = full
        if seed is not None:
            random.seed(seed)
        try:
            with _watch_prints(lines):
                runpy.run_path(os.path.join(REF, VARIANT_FILE[variant]), run_name="__main__")
        except _Hang:
            rec["hang"] = True
        except SystemExit as e:
            rec["exit"] = e.code if isinstance(e.code, int) else 1
        except Exception as e:  # reference crash (e.g. SURVEY Q4: empty reduce)
            rec["exception"] = f"{type(e).__name__}: {e}"
        rec["stdout"] = _normalise(lines)
        if os.path.exists(out_path):
            raw = open(out_path, "rb").read()
            rec["output_sha256"] = hashlib.sha256(raw).hexdigest()
            data = json.loads(raw)
            rec["output_ids"] = [d["id"] for d in data]
            rec["output_colors"] = [d["color"] for d in data]
        if os.path.exists(graph_out):
            raw = open(graph_out, "rb").read()
            rec["graph_out_sha256"] = hashlib.sha256(raw).hexdigest()
            rec["graph_out"] = [[d["id"], d["neighbors"]] for d in json.loads(raw)]
    return rec


def _run_direct(variant, graph_json_path, k=UNBOUNDED_K):
    """Call the reference's graph_coloring directly (unbounded k)."""
    import runpy
    _setup_paths()
    mod = runpy.run_path(os.path.join(REF, VARIANT_FILE[variant]), run_name="golden")
    from graph import Graph  # reference graph.py (on sys.path)
    from pyspark import SparkContext, RDD

    g = Graph(0, 0)
    try:
        nodes = g.deserialize_graph(graph_json_path)
    except Exception as e:  # coloring.py:179-181 path (e.g. KeyError on a missing id)
        return {"k": k, "load_error": f"{type(e).__name__}: {e}"}
    ids = [nd.id for nd in nodes]
    sc = SparkContext()
    rdd = RDD(nodes)  # single partition, file order (coloring.py:201-209)

    snapshots = []
    orig_bc = mod["broadcast_colors"]

    def bc_wrapper(graph_rdd, sc_):
        b = orig_bc(graph_rdd, sc_)
        snapshots.append(dict(b.value))
        return b

    gc_fn = mod["graph_coloring"]
    gc_fn.__globals__["broadcast_colors"] = bc_wrapper
    lines = []
    rec = {"k": k, "hang": False}
    try:
        with _watch_prints(lines):
            ok, out_rdd = gc_fn(rdd, k, sc)
        rec["ok"] = bool(ok)
        final = {nd.id: nd.color for nd in out_rdd.collect()}
        rec["colors"] = [final[i] for i in ids]
        rec["out_order_ids"] = [nd.id for nd in out_rdd.collect()]
    except _Hang:
        rec["hang"] = True
    except Exception as e:
        rec["exception"] = f"{type(e).__name__}: {e}"
    rec["rounds_U"] = [int(ln.split(":")[1]) for ln in lines if ln.startswith("Uncolored nodes remaining")]
    # round in which each vertex is first seen coloured at a round start
    cr = [-1] * len(ids)
    pos = {vid: i for i, vid in enumerate(ids)}
    for r, snap in enumerate(snapshots):
        for vid, c in snap.items():
            i = pos[vid]
            if c != -1 and cr[i] == -1:
                cr[i] = r
    rec["colored_round"] = cr
    rec["n_broadcasts"] = len(snapshots)
    return rec


def _graph_from_ref_generator(n, d, seed):
    _setup_paths()
    from graph import Graph
    random.seed(seed)
    g = Graph(n, d)
    return [[nd.id, [nb.id for nb in nd.neighbors]] for nd in g.nodes]


# ---------------------------------------------------------------------------------------------
# case table
# ---------------------------------------------------------------------------------------------

def _mesh(nx, ny, nz):
    """3-D 7-point mesh, id = x + nx*(y + ny*z), neighbours in order -x,+x,-y,+y,-z,+z."""
    out = []
    for z in range(nz):
        for y in range(ny):
            for x in range(nx):
                nb = []
                for dx, dy, dz in ((-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)):
                    a, b, c = x + dx, y + dy, z + dz
                    if 0 <= a < nx and 0 <= b < ny and 0 <= c < nz:
                        nb.append(a + nx * (b + ny * c))
                out.append([x + nx * (y + ny * z), nb])
    return out


def _custom_cases():
    cases = {}
    cases["self_loop"] = [[5, [5, 7]], [7, [5]]]
    cases["edgeless"] = [[0, []], [1, []], [2, []]]
    cases["single_edge"] = [[0, [1]], [1, [0]]]
    cases["arbitrary_ids"] = [[100, [-3, 42]], [-3, [100, 7]], [42, [100, 7]], [7, [-3, 42, 9]], [9, [7]], [55, []]]
    cases["duplicates"] = [[0, [1, 1, 2]], [1, [0, 0, 2]], [2, [0, 1, 3]], [3, [2]]]
    cases["asymmetric"] = [[0, [1, 2]], [1, [2]], [2, []], [3, [0]]]
    cases["asym_chain"] = [[0, [1]], [1, [2]], [2, [3]], [3, [0, 4]], [4, [3]]]
    cases["cycle6"] = [[i, [(i - 1) % 6, (i + 1) % 6]] for i in range(6)]
    cases["cycle7"] = [[i, [(i + 1) % 7, (i - 1) % 7]] for i in range(7)]
    cases["k5"] = [[i, [j for j in range(5) if j != i]] for i in range(5)]
    cases["star"] = [[0, [1, 2, 3, 4, 5]]] + [[i, [0]] for i in range(1, 6)]
    cases["two_components"] = [[0, [1]], [1, [0, 2]], [2, [1]], [3, [4]], [4, [3, 5]], [5, [4]]]
    cases["triangle_plus_path"] = [[0, [1, 2]], [1, [0, 2]], [2, [0, 1, 3]], [3, [2, 4]], [4, [3]]]
    cases["petersen"] = [[0, [1, 4, 5]], [1, [0, 2, 6]], [2, [1, 3, 7]], [3, [2, 4, 8]], [4, [3, 0, 9]],
                         [5, [0, 7, 8]], [6, [1, 8, 9]], [7, [2, 5, 9]], [8, [3, 5, 6]], [9, [4, 6, 7]]]
    cases["mesh4"] = _mesh(4, 4, 4)
    cases["mesh6x5x4"] = _mesh(6, 5, 4)
    cases["self_loop_only_seed"] = [[0, [0, 0, 0]], [1, [2]], [2, [1]]]
    cases["missing_neighbor"] = [[0, [1]], [1, [0, 99]]]
    return cases


def case_table():
    """name -> dict(kind, graph or params, cli extras)."""
    table = {}
    ref_graph = json.load(open(os.path.join(REF, "graph.json")))
    table["graph_json"] = {"kind": "file", "graph": [[d["id"], d["neighbors"]] for d in ref_graph],
                           "variants": "AB"}
    for name, g in _custom_cases().items():
        table[name] = {"kind": "custom", "graph": g, "variants": "AB"}
    # reference generator, random.seed(s); Graph(n, d)  (graph.py:30-43)
    gens = []
    for n, d in ((10, 3), (20, 5), (50, 3), (50, 5), (100, 10), (200, 5), (200, 10)):
        for s in range(4):
            gens.append((n, d, s))
    for s in range(6):
        gens.append((1000, 8, s))
    for s in (0, 1, 2, 3):
        gens.append((3000, 6, s))
    for s in (0, 1, 2, 3, 4, 5):
        gens.append((10000, 8, s))
    for n, d, s in gens:
        variants = "AB" if n <= 3000 else ("AB" if s == 0 else "A")
        table[f"gen_{n}_{d}_s{s}"] = {"kind": "gen", "params": [n, d, s], "variants": variants}
    # K0 below M: --max-degree smaller than needed (coloring.py:212)
    table["k5_maxdeg2"] = {"kind": "custom", "graph": _custom_cases()["k5"], "variants": "AB",
                           "cli_extra": ["--max-degree", "2"]}
    table["graph_json_maxdeg9"] = {"kind": "file", "graph": table["graph_json"]["graph"], "variants": "AB",
                                   "cli_extra": ["--max-degree", "9"]}
    # CLI generation mode with a seeded global RNG (coloring.py:182-187)
    table["cli_generate_200_5_s7"] = {"kind": "cli_gen", "params": [200, 5, 7], "variants": "AB"}
    return table


def _write_graph_json(graph, path):
    with open(path, "w") as f:
        json.dump([{"id": i, "neighbors": nb, "color": -1} for i, nb in graph], f, indent=4)


def build_case(name):
    spec = case_table()[name]
    t0 = time.time()
    rec = {"name": name, "kind": spec["kind"]}
    if spec["kind"] == "gen":
        n, d, s = spec["params"]
        graph = _graph_from_ref_generator(n, d, s)
        rec["params"] = {"node_count": n, "max_degree": d, "seed": s}
    elif spec["kind"] == "cli_gen":
        n, d, s = spec["params"]
        graph = None
        rec["params"] = {"node_count": n, "max_degree": d, "seed": s}
    else:
        graph = spec["graph"]
    rec["variants"] = {}
    with tempfile.TemporaryDirectory() as td:
        gpath = os.path.join(td, "g.json")
        for v in spec["variants"]:
            vr = {}
            if spec["kind"] == "cli_gen":
                n, d, s = spec["params"]
                vr["cli"] = _run_cli(v, ["--node-count", str(n), "--max-degree", str(d),
                                         "--output-graph", "@GRAPH_OUT", "--output-coloring", "@OUT"], seed=s)
                graph = vr["cli"]["graph_out"]
                del vr["cli"]["graph_out"]
                _write_graph_json(graph, gpath)
            else:
                _write_graph_json(graph, gpath)
                vr["cli"] = _run_cli(v, ["--input", gpath] + spec.get("cli_extra", []) + ["--output-coloring", "@OUT"])
            vr["run"] = _run_direct(v, gpath)
            rec["variants"][v] = vr
    rec["graph"] = graph
    rec["gen_seconds"] = round(time.time() - t0, 2)
    path = os.path.join(OUT_DIR, f"{name}.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(rec, f, separators=(",", ":"))
    return name, rec["gen_seconds"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=6)
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    os.makedirs(OUT_DIR, exist_ok=True)
    names = args.only or list(case_table())
    # slowest first (variant B at n=10^4 is quadratic)
    names.sort(key=lambda s: -int(s.split("_")[1]) if s.startswith("gen_") else 0)
    with mp.get_context("fork").Pool(args.jobs, maxtasksperchild=1) as pool:
        for name, secs in pool.imap_unordered(build_case, names):
            print(f"{name}: {secs}s", flush=True)


if __name__ == "__main__":
    main()
