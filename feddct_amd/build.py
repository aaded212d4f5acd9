"""Build libfedagg.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# fedagg_k*.hip: the reduce kernel variants, split over units that compile
# in parallel (one unit held them all: 5 minutes of device compilation)
SRCS = [os.path.join(HERE, "csrc", f) for f in
        ("fedagg.hip", "fedagg_k1.hip", "fedagg_k2.hip", "fedagg_k2w.hip", "fedagg_k4.hip",
         "prox.hip")]
HEADERS = [os.path.join(HERE, "csrc", "common.h"), os.path.join(HERE, "csrc", "reduce_impl.h"),
           os.path.join(HERE, "..", "include", "fedagg.h")]
DEPS = SRCS + HEADERS
OUT = os.path.join(HERE, "libfedagg.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.environ.get("HIPCC", os.path.join(ROCM, "bin", "hipcc"))
# test infrastructure (build_loopback, below)
LOOP_DIR = os.path.join(HERE, "..", "tests", "loopback")

# -ffp-contract=off: no FMA contraction anywhere (the weighted path's x*w must
# round before the add); no -ffast-math / denormal flushing: the sum must be
# IEEE fp32 round-to-nearest-even with subnormals, like torch's CPU kernel.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall"]


# The multi-GPU exchange (RCCL) is a separate library over libfedagg.so's
# public ABI, so the core library does not depend on RCCL.  librccl.so.1
# resolves to the copy torch has already loaded (same soname).
COMM_SRC = os.path.join(HERE, "csrc", "fedcomm.hip")
COMM_DEPS = [COMM_SRC, os.path.join(HERE, "csrc", "common.h"),
             os.path.join(HERE, "..", "include", "fedagg.h"),
             os.path.join(HERE, "..", "include", "fedagg_comm.h")]
COMM_OUT = os.path.join(HERE, "libfedagg_comm.so")


# The drop-in's per-call host bookkeeping (arena checks, autograd version
# bumps) as a small CPython extension against the running torch (g++; host
# code only).
SHIM_SRC = os.path.join(HERE, "csrc", "shim.cpp")


def shim_path() -> str:
    import sysconfig
    return os.path.join(HERE, "_fa_shim" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_shim(force: bool = False) -> str:
    import sysconfig

    import torch
    from torch.utils.cpp_extension import include_paths
    out = shim_path()
    if not force and not _stale(out, [SHIM_SRC, os.path.join(HERE, "..", "include", "fedagg.h")]):
        return out
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", *("-I" + p for p in include_paths()),
           "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(ROCM, "include"),
           "-D__HIP_PLATFORM_AMD__=1", SHIM_SRC, "-o", out + ".tmp",
           "-L" + tlib, "-ltorch_python", "-lc10", "-lc10_hip", "-ltorch_cpu",
           "-Wl,-rpath," + tlib]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def _stale(out, deps):
    return not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d)
                                                                   for d in deps)


def _compile_units(srcs, flags, jobs=None, force=False):
    """hipcc -c of every stale unit (older than its source or a shared
    header), several at once; returns the object paths."""
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "0")) or os.cpu_count() or 4, 16)
    cflags = [f for f in flags if f not in ("-shared",)]
    objs, procs = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and not _stale(obj, [src] + HEADERS):
            continue
        while len([p for p in procs if p.poll() is None]) >= jobs:
            procs[[p.poll() is None for p in procs].index(True)].wait()
        procs.append(subprocess.Popen([HIPCC, *cflags, "-c", "-o", obj, src]))
    bad = [p.args[-1] for p in procs if p.wait() != 0]
    if bad:
        raise subprocess.CalledProcessError(1, f"hipcc -c {bad}")
    return objs


def build(force: bool = False, extra=()) -> str:
    if force or _stale(OUT, DEPS):
        objs = _compile_units(SRCS, [*FLAGS, *extra], force=force or bool(extra))
        cmd = [HIPCC, *FLAGS, *extra, "-Wl,-soname,libfedagg.so", "-o", OUT + ".tmp", *objs]
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    if force or _stale(COMM_OUT, COMM_DEPS + [OUT]):
        cmd = [HIPCC, *FLAGS, *extra, "-o", COMM_OUT + ".tmp", COMM_SRC, "-L" + HERE, "-lfedagg",
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,$ORIGIN"]
        subprocess.run(cmd, check=True)
        os.replace(COMM_OUT + ".tmp", COMM_OUT)
    build_shim(force)
    build_example(force)
    if os.path.isdir(LOOP_DIR):   # test infrastructure; absent when tests/ is not shipped
        build_loopback(force, extra)
    return OUT


# A native consumer of the C ABI (examples/c_abi_round.cpp): no Python, no
# torch; run by tests/test_gpu_cabi.py.
EXAMPLE_SRC = os.path.join(HERE, "..", "examples", "c_abi_round.cpp")
EXAMPLE_OUT = os.path.join(HERE, "..", "examples", "c_abi_round")


def build_example(force: bool = False) -> str:
    if force or _stale(EXAMPLE_OUT, [EXAMPLE_SRC, OUT, os.path.join(HERE, "..", "include",
                                                                     "fedagg.h")]):
        cmd = [HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17",
               "-I" + os.path.join(HERE, "..", "include"), "-o", EXAMPLE_OUT + ".tmp",
               EXAMPLE_SRC, "-L" + HERE, "-lfedagg", "-Wl,-rpath,$ORIGIN/../feddct_amd"]
        subprocess.run(cmd, check=True)
        os.replace(EXAMPLE_OUT + ".tmp", EXAMPLE_OUT)
    return EXAMPLE_OUT


# Test infrastructure: the native multi-rank rounds on one GPU.  fedcomm.hip
# compiled unchanged, linked against an in-process loopback of the RCCL
# subset it calls (tests/loopback/loopccl.hip) instead of librccl, and a C++
# driver (tests/loopback/loop_round.cpp) run by tests/test_gpu_loopback.py.
# Nothing in the package links or loads these.


def build_loopback(force: bool = False, extra=()) -> str:
    inc = "-I" + os.path.join(HERE, "..", "include")
    ccl_src = os.path.join(LOOP_DIR, "loopccl.hip")
    ccl = os.path.join(LOOP_DIR, "libloopccl.so")
    comm = os.path.join(LOOP_DIR, "libfedagg_comm_loop.so")
    drv_src = os.path.join(LOOP_DIR, "loop_round.cpp")
    drv = os.path.join(LOOP_DIR, "loop_round")
    if force or _stale(ccl, [ccl_src]):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared",
                        "-Wall", "-Wl,-soname,libloopccl.so", "-o", ccl + ".tmp", ccl_src],
                       check=True)
        os.replace(ccl + ".tmp", ccl)
    if force or _stale(comm, COMM_DEPS + [OUT, ccl]):
        subprocess.run([HIPCC, *FLAGS, *extra, "-Wl,-soname,libfedagg_comm_loop.so", "-o", comm + ".tmp",
                        COMM_SRC, "-L" + HERE, "-lfedagg", "-L" + LOOP_DIR, "-lloopccl",
                        "-Wl,-rpath,$ORIGIN:$ORIGIN/../../feddct_amd"], check=True)
        os.replace(comm + ".tmp", comm)
    if force or _stale(drv, [drv_src, comm, os.path.join(HERE, "..", "include", "fedagg_comm.h")]):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", inc, "-o",
                        drv + ".tmp", drv_src, "-L" + HERE, "-lfedagg", "-L" + LOOP_DIR,
                        "-lfedagg_comm_loop", "-lloopccl", "-pthread",
                        "-Wl,-rpath,$ORIGIN:$ORIGIN/../../feddct_amd"], check=True)
        os.replace(drv + ".tmp", drv)
    return drv


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
