#!/bin/bash
# Build libgcolor.so with extra compile-time settings into variants/NAME/ (git-ignored, but it
# travels to the GPU box with the tree): GC_LIB_PATH=variants/NAME/libgcolor.so selects it.
#   bash tools/build_var.sh NAME "-DGC_HUB_REG=0 ..."
set -euo pipefail
NAME=$1; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/distributed-graph-coloring-with-pyspark_amd/csrc" -j8 EXTRA="$FLAGS" \
  OUTDIR="$ROOT/variants/$NAME" OBJDIR="$ROOT/variants/$NAME/obj/" > /dev/null
rm -rf "$ROOT/variants/$NAME/obj"
echo "variants/$NAME/libgcolor.so"
