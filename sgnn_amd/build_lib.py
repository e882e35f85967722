"""Build libsgnn_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels to the GPU box with the repo snapshot)."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libsgnn_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
         "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result"]


# the radius search's translation unit without FMA contraction: its graphs are bit-exact against the
# oracle's `dims summed in order, no contraction` rule (the distance blocks of the other units carry
# `#pragma clang fp contract(off)` as well)
NO_CONTRACT = {"radius.hip"}


def flags_for(src: str):
    f = [x for x in FLAGS if x != "-shared"]
    if os.path.basename(src) in NO_CONTRACT:
        f = ["-ffp-contract=off" if x == "-ffp-contract=fast" else x for x in f]
    return f


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "sgnn.h")]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in deps())


OBJDIR = os.path.join(LIBDIR, "obj")   # per-source objects (git- and gpurun-ignored): incremental rebuilds


def build(force: bool = False, verbose: bool = False, defines=(), lib: str = LIB) -> str:
    """Compile every csrc/*.hip for gfx950 and link `lib`.  `defines` (e.g.
    SGNN_PROBE) are for experiment builds linked to another path.  A source is
    recompiled when it, any header, or this script is newer than its object."""
    if not force and not defines and lib == LIB and not needs_build():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    objs = []
    procs = []
    tag = "".join("_" + d.lower().replace("=", "_") for d in defines)
    headers = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "sgnn.h"), __file__]
    newest_header = max(os.path.getmtime(h) for h in headers)
    for src in sources():
        obj = os.path.join(OBJDIR, os.path.basename(src) + tag + ".o")
        objs.append(obj)
        if (not force and os.path.exists(obj) and os.path.getmtime(obj) > os.path.getmtime(src)
                and os.path.getmtime(obj) > newest_header):
            continue
        cmd = [HIPCC, *flags_for(src), *[f"-D{d}" for d in defines], "-c", src, "-o", obj + ".tmp",
               "-I", os.path.join(ROOT, "include")]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), obj))
    for p, obj in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
        os.replace(obj + ".tmp", obj)
    tmp = lib + ".tmp"
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs])
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
