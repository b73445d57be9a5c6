"""Builds the in-tree HIP/C++ library `antrea_amd/_build/libgpc.so` for gfx950.

    python -m antrea_amd.build          # incremental
    python -m antrea_amd.build --force  # rebuild everything

hipcc cross-compiles the kernel for gfx950 without a GPU; host C++ (compiler.cpp, image.cpp) is
compiled with the same toolchain. The .so is git-ignored but travels to the GPU box in the gpurun
snapshot (it is not listed in .gpurunignore).

Rebuilds are decided by content, not mtime: every object carries a stamp file with the SHA-256 of
its compile command, source and headers, so a snapshot whose sources differ from the ones a
travelling .so was built from is rebuilt, and one that matches is not.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libgpc.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
if ARCH != "gfx950":  # the grouping / un-permute kernels use up to 141 KB of LDS (gfx950: 160 KB)
    raise RuntimeError("libgpc targets gfx950 only (PYTORCH_ROCM_ARCH=%s)" % ARCH)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HOST_SRCS = ["compiler.cpp", "image.cpp", "flowtext.cpp", "service.cpp"]
HIP_SRCS = ["classify.hip", "api.cpp"]
HEADERS = ["model.hpp", "compiler.hpp", "core.hpp", "image.hpp", "launch.hpp", "oplog.hpp", "service.hpp"]
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def _digest(cmd, srcs):
    h = hashlib.sha256(" ".join(cmd).encode())
    for s in srcs:
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(dst, cmd, srcs):
    """True when dst is missing or was built from other inputs (its .sha256 stamp differs)."""
    stamp = dst + ".sha256"
    if not os.path.exists(dst) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(cmd, srcs)


def _stamp(dst, cmd, srcs):
    with open(dst + ".sha256", "w") as f:
        f.write(_digest(cmd, srcs) + "\n")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def build(force: bool = False, verbose: bool = False, variant: str = "", defines=()) -> str:
    """`variant`/`defines`: an experiment build of the kernel (libgpc_<variant>.so, selected at run
    time with GPC_LIB); the default build is the product library."""
    os.makedirs(OUT, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "gpc.h")]
    objs = []
    for s in HOST_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT, s + ".o")
        cmd = ["g++"] + CXXFLAGS + ["-c", src, "-o", obj]
        if force or _stale(obj, cmd, [src] + hdrs):
            _run(cmd)
            _stamp(obj, cmd, [src] + hdrs)
        objs.append(obj)
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        tag = "_" + variant if (variant and s.endswith(".hip")) else ""
        obj = os.path.join(OUT, s + tag + ".o")
        lang = ["-x", "hip"] if s.endswith(".hip") else []
        dfl = ["-D" + d for d in defines] if s.endswith(".hip") else []
        cmd = [HIPCC, "--offload-arch=" + ARCH] + CXXFLAGS + dfl + lang + ["-c", src, "-o", obj]
        if force or _stale(obj, cmd, [src] + hdrs):
            _run(cmd)
            _stamp(obj, cmd, [src] + hdrs)
        objs.append(obj)
    lib = os.path.join(OUT, "libgpc_%s.so" % variant) if variant else LIB
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs
    if force or _stale(lib, cmd, objs):
        _run(cmd)
        _stamp(lib, cmd, objs)
    if verbose:
        print(lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
