"""Build recipe of libarctopk.so (hipcc, gfx950 only; cross-compiles without a GPU).

    python -m allreducetopk_amd.build        # -> allreducetopk_amd/lib/libarctopk.so

The library is built in-tree so it travels with the repo snapshot to the GPU box.

Build integrity: every build embeds ``source_hash()`` -- a SHA-256 over the sources,
the public header, this recipe's compiler flags and any ``-D`` defines -- in the string
``arctopk_version()`` returns.  ``build()`` rebuilds whenever the hash of the tree
differs from the one the library carries, and ``_native.lib()`` refuses a library whose
hash does not match the sources next to it (unless ``ARCTOPK_LIB`` names a library
explicitly, e.g. an A/B tuning variant).
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libarctopk.so")
SOURCES = ["plan.hip", "arctopk_kernels.hip", "sparse_kernels.hip", "mselect.hip", "vdraw.hip",
           "projection.cpp", "step.cpp", "exchange.cpp", "wire.hip"]
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
         "-Wno-unused-function"]
HASH_RE = re.compile(rb"src:([0-9a-f]{16})")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libarctopk)")


def source_hash(defines=()) -> str:
    """16 hex digits of SHA-256 over every file in csrc/, include/arctopk.h, the
    compiler flags and the defines (what determines the built machine code)."""
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if not f.startswith("."))
    for f in files:
        h.update(f.encode() + b"\0")
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(INCLUDE, "arctopk.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join([ARCH, *FLAGS, *sorted(defines)]).encode())
    return h.hexdigest()[:16]


def embedded_hash(path: str = LIB):
    """The source hash a built library carries (read from its bytes; no loading)."""
    try:
        with open(path, "rb") as fh:
            m = HASH_RE.search(fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _stale() -> bool:
    return embedded_hash(LIB) != source_hash()


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """Compile the HIP sources into one shared library (gfx950).  `out` / `defines`
    build tuning variants (e.g. -DARCTOPK_ENC_WAVES=4) next to the product library."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = out + ".tmp"
    digest = source_hash(defines)
    common = [f"--offload-arch={ARCH}", *FLAGS, *[f"-D{d}" for d in defines],
              f'-DARCTOPK_SRC_HASH="{digest}"', f"-I{INCLUDE}", f"-I{CSRC}"]
    objdir = tmp + ".objs"
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s_) + ".o") for s_ in srcs]
    # one compiler process per source (the kernels file dominates; the others overlap it)
    cmds = [[hipcc(), *[f for f in common if f != "-shared"], "-c", s_, "-o", o]
            for s_, o in zip(srcs, objs)]
    if verbose:
        for c in cmds:
            print(" ".join(c), file=sys.stderr)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(jobs) as ex:
        for r in ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds):
            if r.returncode:
                raise subprocess.CalledProcessError(r.returncode, r.args, r.stdout, r.stderr + "\n" + r.stdout)
            if verbose and r.stderr:
                print(r.stderr, file=sys.stderr)
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", tmp], check=True)
    shutil.rmtree(objdir, ignore_errors=True)
    os.replace(tmp, out)
    return out

if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
