#!/bin/bash
# Build libgcolor.so with extra compile-time settings into build_variants/NAME/ (for A/B
# runs: GC_LIB_PATH=build_variants/NAME/libgcolor.so python bench.py ...).
#   bash tools/build_variant.sh NAME "-DGC_CSLOTS=1 ..."
set -euo pipefail
NAME=$1; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/distributed-graph-coloring-with-pyspark_amd/csrc" -j8 EXTRA="$FLAGS" \
  OUTDIR="$ROOT/build_variants/$NAME" OBJDIR="$ROOT/build_variants/$NAME/obj/" > /dev/null
rm -rf "$ROOT/build_variants/$NAME/obj"
echo "$ROOT/build_variants/$NAME/libgcolor.so"
