"""Literal emulation of the reference's outer colour-count loop (coloring.py:211-235).

TEST HELPER. Drives a *bounded* colouring function attempt by attempt, exactly as the
reference does (k = K0, K0-1, ... until the first failure), and produces the stdout
transcript (timing lines normalised) and the colouring written to --output-coloring.
Used to pin (a) the oracle's bounded-k semantics against the recorded reference CLI
runs and (b) the product CLI's single-run derivation of the same transcript.
"""


def validate_lines(unc, conf):
    """validate_graph_coloring prints (coloring.py:149-162) + the caller's print (:224)."""
    if unc > 0:
        return [f"Graph coloring failed: {unc} nodes have no colors.", "Validation result: False"]
    if conf > 0:
        return [f"Graph coloring failed: {conf} conflicts detected.", "Validation result: False"]
    return ["Validation result: True"]


def emulate(color_fn, validate_fn, K0, max_attempts=10_000):
    """color_fn(k) -> dict(status, colors, round_U, fail_count); validate_fn(colors)->(u,c)."""
    lines = []
    k = K0
    final = None
    for _ in range(max_attempts):
        res = color_fn(k)
        lines += [f"Uncolored nodes remaining: {u}" for u in res["round_U"]]
        failed = res["status"] == 1
        if failed:
            lines.append(f"Graph coloring failed: {res['fail_count']} nodes have no available colors.")
        lines.append(f"Number of colors: {k}")
        lines.append("Iteration time: <t> seconds")
        lines += validate_lines(*validate_fn(res["colors"]))
        final = res["colors"]
        if failed:
            lines.append("Total execution time: <t> seconds")
            lines.append(f"Minimal number of colors: {k + 1}")
            return lines, list(final)
        k -= 1
    raise RuntimeError("reference k-loop does not terminate on this input")
