"""coloring.py-compatible command line (coloring.py:165-243, coloring_optimized.py:233-311).

Same flags, stdout lines, exit codes and JSON files as the reference.  Additive flags:
``--variant {A,B}`` (A = coloring.py, B = coloring_optimized.py), ``--seed`` (seeds
Python's ``random`` before generation so ``Graph(N, D)`` is reproducible),
``--compat-output`` (write the reference's exact output file, see below), ``--no-e1``,
``--device``.  ``--input`` also takes a binary CSR file (``.gcsr``, detected by its magic
bytes) and ``--output-graph x.gcsr`` writes one.

The reference decrements k from K0 and reruns the whole colouring until an attempt fails
(coloring.py:211-231).  Attempt k is the unbounded run cut at the first round whose
largest proposal is >= k (verified on the golden set), so the engine
runs ONE unbounded colouring and at most ONE bounded attempt (the failing one) and
derives the reference's transcript from them.

Output file: by default the valid colouring of the last successful attempt (== the
unbounded run, every output passes validation); ``--compat-output`` writes what the
reference writes -- the failed attempt's round-start snapshot, with -1 entries.
"""
import argparse
import random
import sys
import time

import numpy as np

from . import graphio
from .generators import reference_csr


def attempt_plan(K0, round_maxmex, max_color):
    """(successful attempts k list, failing k or None, minimal colours printed)."""
    top = max((int(m) for m in round_maxmex), default=-1)
    if top >= 0:
        fail_k = K0 if K0 <= top else top
    else:
        fail_k = None
    if fail_k is not None:
        ok_ks = list(range(K0, fail_k, -1))
        minimal = fail_k + 1
    else:  # nothing can fail: the reference loops forever; stop at the colours used
        stop = max(int(max_color) + 1, 1)
        ok_ks = list(range(K0, stop - 1, -1)) if K0 >= stop else [K0]
        minimal = stop
    return ok_ks, fail_k, minimal


def validate_lines(uncolored, conflicts):
    """validate_graph_coloring's prints (coloring.py:149-162) + coloring.py:224."""
    if uncolored > 0:
        return [f"Graph coloring failed: {uncolored} nodes have no colors.", "Validation result: False"]
    if conflicts > 0:
        return [f"Graph coloring failed: {conflicts} conflicts detected.", "Validation result: False"]
    return ["Validation result: True"]


def transcript(K0, full, full_ms, full_val, bounded=None, bounded_ms=0.0, bounded_val=None):
    """Reference stdout for the k-loop, from one unbounded run (+ the failing attempt).

    ``full``/``bounded`` need: round_U, round_maxmex, max_color (+ fail_count for bounded).
    Returns (lines, fail_k, minimal)."""
    ok_ks, fail_k, minimal = attempt_plan(K0, full.round_maxmex, full.max_color)
    lines = []
    for k in ok_ks:
        lines += [f"Uncolored nodes remaining: {int(u)}" for u in full.round_U]
        lines.append(f"Number of colors: {k}")
        lines.append(f"Iteration time: {full_ms / 1000.0:.2f} seconds")
        lines += validate_lines(*full_val)
    if fail_k is not None:
        lines += [f"Uncolored nodes remaining: {int(u)}" for u in bounded.round_U]
        lines.append(f"Graph coloring failed: {int(bounded.fail_count)} nodes have no available colors.")
        lines.append(f"Number of colors: {fail_k}")
        lines.append(f"Iteration time: {bounded_ms / 1000.0:.2f} seconds")
        lines += validate_lines(*bounded_val)
    return lines, fail_k, minimal


def build_parser():
    p = argparse.ArgumentParser(description="Graph Coloring CLI")
    p.add_argument("--input", type=str, help="Input graph file (JSON, or binary .gcsr)")
    p.add_argument("--node-count", type=int, help="Number of nodes for graph generation")
    p.add_argument("--max-degree", type=int, help="Maximum degree for graph generation")
    p.add_argument("--output-graph", type=str, help="Output file to serialize the generated graph")
    p.add_argument("--output-coloring", type=str, required=True, help="Output file for coloring results")
    # additive flags (no reference counterpart)
    p.add_argument("--variant", choices=["A", "B"], default="A",
                   help="A = coloring.py semantics (default), B = coloring_optimized.py")
    p.add_argument("--seed", type=int, default=None, help="random.seed() before Graph(node_count, max_degree)")
    p.add_argument("--compat-output", action="store_true",
                   help="write the reference's failed-attempt snapshot instead of the valid colouring")
    p.add_argument("--no-e1", action="store_true", help="disable the stall re-seed extension (E1)")
    p.add_argument("--device", type=int, default=None, help="GPU ordinal")
    p.add_argument("--native-gen", action="store_true",
                   help="generate with the native generator (graph.py:30-43's process on a splitmix64 stream seeded "
                        "by --seed) instead of Python's random -- for node counts past what Python can build")
    p.add_argument("--priority-seed", type=int, default=None,
                   help="variant A: order each colour's conflict resolution by the seeded priority "
                        "prio_hash(seed, v) instead of the reference's (deg, pos)")
    p.add_argument("--speculative", action="store_true",
                   help="variant A: speculative first-fit rounds with one-shot resolution (not the reference's "
                        "semantics; valid colourings)")
    return p


def main(argv=None, out=None):
    out = out or sys.stdout

    def say(line):
        print(line, file=out)

    parser = build_parser()
    args = parser.parse_args(argv)
    # Load or generate graph (coloring.py:174-187)
    if args.input:
        try:
            ids, rp, col, symmetric = graphio.load_graph_ex(args.input)
        except Exception as e:  # same message and status as coloring.py:179-181
            say(f"Error loading graph: {e}")
            sys.exit(1)
    else:
        if not args.node_count or not args.max_degree:
            parser.error("--node-count and --max-degree are required when not using --input")
        if args.native_gen:  # graph.py:30-43's process on a splitmix64 stream (gc_gen_uniform), any size
            from .engine import uniform_csr
            rp, col = uniform_csr(args.node_count, args.max_degree, 0 if args.seed is None else args.seed)
            ids = np.arange(args.node_count, dtype=np.int64)
        else:
            if args.seed is not None:
                random.seed(args.seed)
            rp, col = reference_csr(args.node_count, args.max_degree)
            ids = list(range(args.node_count))
        symmetric = True  # the generator links both ends
        if args.output_graph:
            if args.output_graph.endswith(".gcsr"):  # binary CSR
                graphio.write_csr(args.output_graph, rp, col, symmetric=True)
            else:
                graphio.write_graph_json(args.output_graph, ids, rp, col)

    from .engine import DeviceGraph  # the HIP library; fails loudly without it
    if args.device is not None:
        from . import _native
        _native.check("gc_set_device", _native.load().gc_set_device(args.device))
    n = len(ids)
    dg = DeviceGraph.from_csr(rp, col, symmetric=symmetric)
    maxdeg = int((rp[1:] - rp[:-1]).max()) if n else 0
    K0 = args.max_degree + 1 if args.max_degree else maxdeg + 1   # coloring.py:212
    e1 = not args.no_e1

    total_start = time.time()
    t0 = time.time()
    if args.variant == "B" and (args.priority_seed is not None or args.speculative):
        parser.error("--priority-seed and --speculative apply to variant A")
    mode = dict(priority=args.priority_seed, speculative=args.speculative)
    full = dg.color(args.variant, e1=e1, **mode)
    full_ms = (time.time() - t0) * 1000.0
    if full.status == 2:
        # E1 disabled and the reference would spin forever here (coloring.py:93-95)
        for u in full.round_U:
            say(f"Uncolored nodes remaining: {int(u)}")
        say("Graph coloring stalled: no uncoloured vertex has a coloured neighbour (re-run without --no-e1).")
        sys.exit(3)
    full_val = dg.validate(full.colors)
    ok_ks, fail_k, _ = attempt_plan(K0, full.round_maxmex, full.max_color)
    bounded, bounded_ms, bounded_val = None, 0.0, None
    if fail_k is not None:
        t0 = time.time()
        bounded = dg.color(args.variant, num_colors=fail_k, e1=e1, **mode)
        bounded_ms = (time.time() - t0) * 1000.0
        bounded_val = dg.validate(bounded.colors)
    lines, fail_k, minimal = transcript(K0, full, full_ms, full_val, bounded, bounded_ms, bounded_val)
    for ln in lines:
        say(ln)
    say(f"Total execution time: {time.time() - total_start:.2f} seconds")
    say(f"Minimal number of colors: {minimal}")

    final = bounded.colors if (args.compat_output and bounded is not None) else full.colors
    graphio.write_coloring_json(args.output_coloring, ids, final)
    dg.close()
    return 0
