#!/bin/bash
# Host-code sanitizer run: the CPU test
# suite (pytest -m "not gpu") against builds whose HOST code is compiled with
# AddressSanitizer + UndefinedBehaviorSanitizer:
#   - feddct_amd/_fa_shim (csrc/shim.cpp: CPython refcounts, capsules, raw
#     pointers on every drop-in call), built with clang++ instead of g++;
#   - libfedagg.so and libfedagg_comm.so: hipcc with the sanitizers on the
#     host side only (-Xarch_host), so the tile planner (fa_plan_build_host,
#     the balanced / tail-split cuts), the ABI's argument checks and the
#     multi-GPU schedule builder (fa_describe_round, fa_multi_select) run
#     instrumented; the device code is the shipped code (GPU sanitizers are
#     not available on this pool, and no CPU test launches a kernel).
# Everything happens in a scratch copy of the tree ($SAN_DIR, default
# /tmp/fa_san): the repository's own libraries are not touched.  The clang
# ASan runtime is preloaded into the (uninstrumented) Python.  UBSan aborts on
# the first finding; ASan leak checking is off (CPython and torch keep
# allocations alive at exit by design).
#   bash tools/sanitize.sh [pytest args]   -> $SAN_DIR/pytest_san.log
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=${SAN_DIR:-/tmp/fa_san}
LLVM=/opt/rocm/lib/llvm
RT=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
rm -rf "$W"
mkdir -p "$W"
tar -C "$ROOT" --exclude=./.git --exclude=./gpurun_out --exclude='*.so' \
    --exclude=./feddct_amd/build --exclude=__pycache__ -cf - . | tar -C "$W" -xf -
PY_INC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
EXT=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
TLIB=$(python3 -c 'import os, torch; print(os.path.join(os.path.dirname(torch.__file__), "lib"))')
TINC=$(python3 -c 'from torch.utils.cpp_extension import include_paths; print(" ".join("-I" + p for p in include_paths()))')
ABI=$(python3 -c 'import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))')
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-omit-frame-pointer"
cd "$W/feddct_amd"
mkdir -p build
pids=()
for u in fedagg fedagg_k1 fedagg_k2 fedagg_k2w fedagg_k4 prox; do
  hipcc $FLAGS $HSAN -c -o build/$u.o csrc/$u.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
hipcc $FLAGS $HSAN -shared -shared-libsan -Wl,-soname,libfedagg.so -o libfedagg.so build/*.o
hipcc $FLAGS $HSAN -shared -shared-libsan -o libfedagg_comm.so csrc/fedcomm.hip -L. -lfedagg \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,'$ORIGIN'
$LLVM/bin/clang++ -O1 -g -std=c++17 -shared -fPIC -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libsan \
    -D_GLIBCXX_USE_CXX11_ABI=$ABI $TINC -I"$PY_INC" -I/opt/rocm/include -D__HIP_PLATFORM_AMD__=1 \
    csrc/shim.cpp -o _fa_shim$EXT -L"$TLIB" -ltorch_python -lc10 -lc10_hip -ltorch_cpu \
    -Wl,-rpath,"$TLIB"
cd "$W"
# every library the suite loads from this tree must be the instrumented one
for f in feddct_amd/libfedagg.so feddct_amd/libfedagg_comm.so feddct_amd/_fa_shim$EXT; do
  nm -D "$f" | grep __asan_ > /dev/null || { echo "not instrumented: $f"; exit 1; }
done
export ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:detect_odr_violation=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# build() of the oracle's C restatement is not part of this run (plain gcc)
set +e
LD_PRELOAD="$RT" python3 -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@" \
    > "$W/pytest_san.log" 2>&1
rc=$?
set -e
# what that process family had loaded: the instrumented libraries of this
# tree and the ASan runtime
LD_PRELOAD="$RT" python3 - >> "$W/pytest_san.log" 2>&1 <<'PY'
import feddct_amd._lib, feddct_amd.comm as c, feddct_amd._fa_shim  # noqa: F401
c.lib()
maps = open("/proc/self/maps").read().split("\n")
seen = sorted({ln.split()[-1] for ln in maps if ("fedagg" in ln or "fa_shim" in ln
                                                or "asan" in ln) and "/" in ln})
print("loaded:", *seen, sep="\n  ")
PY
tail -12 "$W/pytest_san.log"
grep -E "ERROR: AddressSanitizer|runtime error:" "$W/pytest_san.log" | head -20 || true
exit $rc
