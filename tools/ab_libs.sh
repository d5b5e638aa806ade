#!/bin/bash
# A/B of compile-time variants of libgcolor.so: one process per (variant, cycle), the
# variants alternated over CYCLES cycles (base, v1, v2, base, v1, v2, ...), each process
# timing REPS §8d steps of WORKLOAD with tools/ab_steps.py.  A variant is NAME=PATH to its
# libgcolor.so (PATH "-" = the in-tree build).  Summary: every process's median per variant.
#   bash tools/ab_libs.sh WORKLOAD REPS CYCLES NAME=PATH ...
set -uo pipefail
WL=$1; REPS=$2; CYC=$3; shift 3
for c in $(seq 1 "$CYC"); do
  for spec in "$@"; do
    name=${spec%%=*}; path=${spec#*=}
    if [ "$path" = "-" ]; then
      timeout -k 10 300 python -u tools/ab_steps.py "$WL" "$REPS" "$name=" || exit $?
    else
      GC_LIB_PATH="$path" timeout -k 10 300 python -u tools/ab_steps.py "$WL" "$REPS" "$name=" || exit $?
    fi
  done
done
