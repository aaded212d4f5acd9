#!/bin/bash
# Build a libfedagg.so variant for tools/ab_lib.py: every unit of the library
# recompiled with extra -D flags (the launch rules live in fedagg.hip, the
# kernel instances in fedagg_k*.hip).  Run HERE (CPU); the .so travels to the
# box with the tree (tools/*.so is git-ignored only).
#   bash tools/lib_variant.sh TAG -DFA_TGPU_LOOP_DEPTH=2 ...
#   -> tools/libfedagg_TAG.so
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1; shift
O=feddct_amd/build/variant_$tag
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall"
mkdir -p "$O"
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from feddct_amd import build as b; print(' '.join(b.SRCS))")
pids=()
for s in $srcs; do
  /opt/rocm/bin/hipcc $F "$@" -c -o "$O/$(basename "$s").o" "$s" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc $F -shared -Wl,-soname,libfedagg.so -o "tools/libfedagg_$tag.so" "$O"/*.o
echo "tools/libfedagg_$tag.so"
