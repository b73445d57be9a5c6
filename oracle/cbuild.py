"""Builds oracle/_build/libovs_cls.so from oracle/ovs_cls.c (test infrastructure)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libovs_cls.so")


def build(force=False):
    src = os.path.join(HERE, "ovs_cls.c")
    os.makedirs(OUT, exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-std=c11", "-shared", "-fPIC", "-pthread", src, "-o", LIB], check=True)
    return LIB
