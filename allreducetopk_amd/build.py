"""Build recipe of libarctopk.so (hipcc, gfx950 only; cross-compiles without a GPU).

    python -m allreducetopk_amd.build        # -> allreducetopk_amd/lib/libarctopk.so

The library is built in-tree so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libarctopk.so")
SOURCES = ["plan.hip", "arctopk_kernels.hip", "sparse_kernels.hip", "mselect.hip", "projection.cpp"]
ARCH = "gfx950"


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libarctopk)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, "arctopk.h"),
                                                              os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """Compile the HIP sources into one shared library (gfx950).  `out` / `defines`
    build tuning variants (e.g. -DARCTOPK_ENC_WAVES=4) next to the product library."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines], f"-I{INCLUDE}", f"-I{CSRC}",
           *srcs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
