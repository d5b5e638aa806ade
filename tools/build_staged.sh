#!/bin/bash
# (Re)build every staged compile-time variant of libgcolor.so into build_variants/NAME/ (git-ignored,
# travels with gpurun), so a GPU session can A/B them with GC_LIB_PATH=build_variants/NAME/libgcolor.so
# (DESIGN §11).  Run on the CPU before the session; the flags of each variant are the record.
#   bash tools/build_staged.sh            # every variant
#   bash tools/build_staged.sh NAME ...   # only these
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
declare -A FLAGS=(
  [hinhoist]="-DGC_HIN_HOIST=1"                        # k_hin_fill: hub-index lookups before the hin_col stores
  [marks4]="-DGC_MARK_SLOTS=4"                         # hub-bitmap pushes / in-row claims 4 entries per thread and step
  [claim4]="-DGC_CLAIM_HOIST=1 -DGC_CSLOTS=4"          # k_commit: every slot's claim word before the atomics, 4 slots
  [tile8]="-DGC_TILE_PER=8"                            # merge-path tiles of 8 rows per thread
  [close_call]="-DGC_CLOSE_INLINE=0 -DGC_CLOSE_BATCH=0" # the round close as a call (rounds 1-2: scratch in k_commit)
  [close_interleaved]="-DGC_CLOSE_BATCH=0"             # the round close as rounds 1-3 ran it (store, load, store, ...)
  [all4]="-DGC_HIN_HOIST=1 -DGC_MARK_SLOTS=4 -DGC_CLAIM_HOIST=1"  # every default-off candidate together
  [checks]="-DGC_CHECKS=1"                             # range checks in k_commit (fault hunts)
)
NAMES=("$@")
[ ${#NAMES[@]} -eq 0 ] && NAMES=(hinhoist marks4 claim4 tile8 close_call close_interleaved all4 checks)
for n in "${NAMES[@]}"; do
  [ -n "${FLAGS[$n]+x}" ] || { echo "unknown variant $n" >&2; exit 2; }
  bash "$ROOT/tools/build_variant.sh" "$n" "${FLAGS[$n]}"
done
