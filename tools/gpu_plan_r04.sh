#!/bin/bash
# Round 4's GPU sessions, one gpurun call each (<= 1200 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_plan_r04.sh a
#   a: the stage-overflow corner first (round 3's k_commit fault, fixed by GC_COUNT_MASK and
#      now bounded by the list capacity in every build), then every GPU test, smoke, the
#      bench line with its rocprofv3 trace + FETCH/WRITE PMC passes (profiles/pmc of THIS
#      build), and the hubs-off asynchronous JP that faulted in round 3, last
set -uo pipefail
cd "$(dirname "$0")/.."
case ${1:-} in
  a) exec_steps=(staged:overflow_tree staged:under_ticket_close tests smoke profile:rmat24 staged:async_jp_without_hubs) ;;
  *) echo "usage: $0 a" >&2; exit 2 ;;
esac
bash tools/gpu_session.sh "r04$1" "${exec_steps[@]}"
