#!/bin/bash
# Build a libfedagg.so variant for tools/ab_lib.py: fedagg.hip recompiled
# with extra -D flags, linked with the tree's other objects (the kernel
# instantiation units do not read these flags).  Run HERE (CPU), after
# `python -c "from feddct_amd import build; build.build()"`; the .so travels
# to the box with the tree (tools/*.so is git-ignored only).
#   bash tools/lib_variant.sh TAG -DFA_TGPU_LOOP_DEPTH=2 ...
#   -> tools/libfedagg_TAG.so
set -euo pipefail
cd "$(dirname "$0")/.."
tag=$1; shift
B=feddct_amd/build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall"
mkdir -p "$B/variant_$tag"
/opt/rocm/bin/hipcc $F "$@" -c -o "$B/variant_$tag/fedagg.hip.o" feddct_amd/csrc/fedagg.hip
objs=$(python3 -c "import os, sys; sys.path.insert(0, '.'); from feddct_amd import build as b; print(' '.join('$B/' + os.path.basename(s) + '.o' for s in b.SRCS[1:]))")
/opt/rocm/bin/hipcc $F -shared -Wl,-soname,libfedagg.so -o "tools/libfedagg_$tag.so" \
  "$B/variant_$tag/fedagg.hip.o" $objs
echo "tools/libfedagg_$tag.so"
