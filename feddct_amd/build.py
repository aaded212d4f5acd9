"""Build libfedagg.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f) for f in ("fedagg.hip", "prox.hip")]
DEPS = SRCS + [os.path.join(HERE, "csrc", "common.h"),
               os.path.join(HERE, "..", "include", "fedagg.h")]
OUT = os.path.join(HERE, "libfedagg.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: no FMA contraction anywhere (the weighted path's x*w must
# round before the add); no -ffast-math / denormal flushing: the sum must be
# IEEE fp32 round-to-nearest-even with subnormals, like torch's CPU kernel.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall"]


def build(force: bool = False, extra=()) -> str:
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(
            os.path.getmtime(d) for d in DEPS):
        return OUT
    cmd = [HIPCC, *FLAGS, *extra, "-o", OUT + ".tmp", *SRCS]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
