#!/bin/bash
# (Re)build every staged compile-time variant of libgcolor.so into build_variants/NAME/ (git-ignored,
# travels with gpurun), so a GPU session can A/B them with GC_LIB_PATH=build_variants/NAME/libgcolor.so
# (DESIGN §11).  Run on the CPU before the session; the flags of each variant are the record.
#   bash tools/build_staged.sh            # every variant
#   bash tools/build_staged.sh NAME ...   # only these
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
declare -A FLAGS=(
  [tile16]="-DGC_TILE_PER=16"                          # merge-path tiles of 16 entries per thread (round 3's default)
  [close_call]="-DGC_CLOSE_INLINE=0 -DGC_CLOSE_BATCH=0" # the round close as a call (rounds 1-2: scratch in k_commit)
  [close_interleaved]="-DGC_CLOSE_BATCH=0"             # the round close as rounds 1-3 ran it (store, load, store, ...)
  [checks]="-DGC_CHECKS=1"                             # range checks in k_commit (fault hunts)
  [pushwg]="-DGC_PUSH_BIG_WG=1"                        # long hub-list pushes a workgroup per winner (round 3)
)
NAMES=("$@")
[ ${#NAMES[@]} -eq 0 ] && NAMES=(tile16 close_call close_interleaved checks pushwg)
for n in "${NAMES[@]}"; do
  [ -n "${FLAGS[$n]+x}" ] || { echo "unknown variant $n" >&2; exit 2; }
  bash "$ROOT/tools/build_variant.sh" "$n" "${FLAGS[$n]}"
done
