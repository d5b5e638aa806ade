#!/bin/bash
# Round 4's first GPU sessions, one gpurun call each (<= 1200 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_plan_r04.sh a
# then b, c, d.  Run `bash tools/build_staged.sh` on the CPU first (part d loads its variants).
#   a: the default build -- GPU tests, smoke, the ticket-close corner (default path first), the
#      bench line, the launch-gap microbenchmark and the per-round cost by frontier size
#   b: staged paths I (resume / hybrid, k_commit_big closing the round, rounds replayed as hipGraphs)
#   c: staged paths II (variant B's asynchronous fold, the asynchronous first sweep, small-round grids)
#   d: per-graph pass timing, the combined variant through the hub and parity suites, step
#      timings; the hubs-off asynchronous JP (the path that faulted in round 3) last
set -uo pipefail
cd "$(dirname "$0")/.."
case ${1:-} in
  a) exec_steps=(tests smoke staged:overflow_tree staged:under_ticket_close bench:rmat24 ubench:launch_gap rounds:rmat24) ;;
  b) exec_steps=("staged:resume~or~hybrid" staged:validate_c8 staged:big_close staged:test_graphs_) ;;
  c) exec_steps=(staged:b_async staged:async_resolve staged:small_grid) ;;
  d) exec_steps=(env:GC_PREP_TIMING=1 step:rmat26 env:GC_PREP_TIMING= env:GC_LIB_PATH=build_variants/all4/libgcolor.so
                 file:tests/test_gpu_hubs.py file:tests/test_gpu_parity.py step:rmat26 step:rmat24 step:mesh512
                 env:GC_LIB_PATH= staged:async_jp_without_hubs) ;;
  *) echo "usage: $0 a|b|c|d" >&2; exit 2 ;;
esac
bash tools/gpu_session.sh "r04$1" "${exec_steps[@]}"
