"""Builds the in-tree HIP/C++ library `antrea_amd/_build/libgpc.so` for gfx950.

    python -m antrea_amd.build          # incremental
    python -m antrea_amd.build --force  # rebuild everything

hipcc cross-compiles the kernel for gfx950 without a GPU; host C++ (compiler.cpp, image.cpp) is
compiled with the same toolchain. The .so is git-ignored but travels to the GPU box in the gpurun
snapshot (it is not listed in .gpurunignore).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libgpc.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HOST_SRCS = ["compiler.cpp", "image.cpp", "flowtext.cpp", "service.cpp"]
HIP_SRCS = ["classify.hip", "api.cpp"]
HEADERS = ["model.hpp", "compiler.hpp", "core.hpp", "image.hpp", "launch.hpp", "service.hpp"]
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def _newer(dst, srcs):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in srcs)


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
        if force or _newer(obj, [src] + hdrs):
            _run(["g++"] + CXXFLAGS + ["-c", src, "-o", obj])
        objs.append(obj)
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        tag = "_" + variant if (variant and s.endswith(".hip")) else ""
        obj = os.path.join(OUT, s + tag + ".o")
        if force or _newer(obj, [src] + hdrs):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            dfl = ["-D" + d for d in defines] if s.endswith(".hip") else []
            _run([HIPCC, "--offload-arch=" + ARCH] + CXXFLAGS + dfl + lang + ["-c", src, "-o", obj])
        objs.append(obj)
    lib = os.path.join(OUT, "libgpc_%s.so" % variant) if variant else LIB
    if force or _newer(lib, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs)
    if verbose:
        print(lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
