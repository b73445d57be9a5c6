"""Loader for the TEST-ONLY host emulation library (tests/csrc/emu.cpp)."""
import ctypes as C
import os
import subprocess

import numpy as np

from antrea_amd import gpc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libgpc_emu.so")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(HERE, "csrc", "emu.cpp")
    core = os.path.join(ROOT, "antrea_amd", "csrc", "core.hpp")
    os.makedirs(OUT, exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(src), os.path.getmtime(core)):
        # built under a private name and renamed into place: parallel test workers that rebuild at
        # the same time never load a half-written library
        tmp = "%s.%d.tmp" % (LIB, os.getpid())
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "antrea_amd", "csrc"), src, "-o", tmp], check=True)
        os.replace(tmp, LIB)
    _lib = C.CDLL(LIB)
    _lib.gpc_emu_stats_arr = (C.c_ulonglong * 16).in_dll(_lib, "gpc_emu_stats")
    _lib.gpc_emu_site_arr = (C.c_ulonglong * 2048).in_dll(_lib, "gpc_emu_site_lines")
    _lib.emu_classify.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                  C.POINTER(gpc.gpc_pkt_soa), C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]
    _lib.emu_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(gpc.gpc_pkt_soa), C.c_void_p,
                               C.POINTER(gpc.gpc_trace_step), C.POINTER(C.c_uint32)]
    _lib.emu_classify6.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(gpc.gpc_pkt_soa),
                                   C.c_size_t, C.c_void_p, C.c_void_p]
    return _lib


class _Counters:
    """The kernels accumulate {packets, bytes, non-session packets} per slot (core.hpp count_stage);
    the library publishes {packets, bytes, sessions} (api.cpp fold_counters). The emulation runs the
    same count_stage into a raw array, added to the caller's array in the published format."""

    def __init__(self, counters):
        self.out = counters
        self.raw = None
        if counters is not None:
            assert counters.dtype == np.uint64 and counters.flags.c_contiguous
            self.raw = np.zeros_like(counters)

    @property
    def ptr(self):
        return None if self.raw is None else self.raw.ctypes.data

    def publish(self):
        if self.raw is None:
            return
        r = self.raw.reshape(-1, 3)
        o = self.out.reshape(-1, 3)
        o[:, 0] += r[:, 0]
        o[:, 1] += r[:, 1]
        o[:, 2] += r[:, 0] - r[:, 2]


def classify6(clf: "gpc.Classifier", cols, counters=None):
    """Emulated IPv6 verdicts (n, 2) of the IPv6 image last committed by `clf`."""
    blob, nw, hdr = clf.debug_image6()
    assert blob, "no IPv6 image (ipv6 disabled, or the IPv6 rule set was rejected)"
    soa, keep, n = gpc.pkt_soa_host(cols)
    out = np.zeros(2 * n, dtype=gpc.VERDICT_DTYPE)
    cnt = _Counters(counters)
    pool, _, jhdr = clf.debug_epoch6()
    load().emu_classify6(blob, hdr, pool, jhdr, C.byref(soa), n, out.ctypes.data, cnt.ptr)
    cnt.publish()
    return out.reshape(n, 2)


def classify(clf: "gpc.Classifier", cols, counters=None, lb=None):
    """Emulated verdicts (n, 2) of the image last committed by `clf` (commit may fail with EDEV
    on a host without GPU: the host image is built before the upload). `counters`: optional
    uint64 array of n_slots x 3 {packets, bytes, sessions} accumulated like the kernel does.
    `lb`: optional gpc.LB_DTYPE array of n entries receiving the Service stage results."""
    blob, nw, hdr, _ = clf.debug_image()
    pool, _, jhdr = clf.debug_epoch()
    soa, keep, n = gpc.pkt_soa_host(cols)
    out = np.zeros(2 * n, dtype=gpc.VERDICT_DTYPE)
    cnt = _Counters(counters)
    svc = clf.debug_service_image()
    lptr = None
    if lb is not None:
        assert lb.dtype == gpc.LB_DTYPE and len(lb) >= n
        lptr = lb.ctypes.data
    load().emu_classify(blob, hdr, pool, jhdr, svc, C.byref(soa), n, out.ctypes.data, lptr, cnt.ptr)
    cnt.publish()
    return out.reshape(n, 2)


def commit_host(clf: "gpc.Classifier", full=False):
    """gpc_commit (gpc_compact with full=True) that tolerates the missing device (the host image
    and overlay are still built)."""
    rc = (clf.lib.gpc_compact if full else clf.lib.gpc_commit)(clf.h)
    if rc not in (0, -gpc.GPC_EDEV):
        raise gpc.GpcError(rc, "gpc_commit")


def stats(reset=False):
    arr = load().gpc_emu_stats_arr
    v = list(arr)
    if reset:
        for i in range(16):
            arr[i] = 0
    return v


def site_lines(reset=False):
    arr = load().gpc_emu_site_arr
    v = {i: arr[i] for i in range(2048) if arr[i]}
    if reset:
        for i in range(2048):
            arr[i] = 0
    return v


def snapshot(clf: "gpc.Classifier"):
    """Owned copies of the committed epoch's host state (base image, header, journal pool and
    header offset, Service image): classify_snapshot emulates exactly that epoch later, whatever
    has been committed since. Call it from the thread that commits, right after gpc_commit."""
    blob, nw, hdr, hb = clf.debug_image()
    pool, pw, jhdr = clf.debug_epoch()
    svc = clf.debug_service_image()
    copy = lambda ptr, n, dt: np.ctypeslib.as_array(C.cast(ptr, C.POINTER(dt)), shape=(n,)).copy() if ptr and n else None
    snap = {"blob": copy(blob, nw, C.c_uint32), "hdr": copy(hdr, hb, C.c_uint8),
            "pool": copy(pool, pw, C.c_uint32), "jhdr": jhdr, "svc": None}
    assert not svc, "epochs with a Service image are not snapshotted"
    return snap


def classify_snapshot(snap, cols, counters=None):
    """Emulated verdicts (n, 2) of a snapshot() epoch."""
    soa, keep, n = gpc.pkt_soa_host(cols)
    out = np.zeros(2 * n, dtype=gpc.VERDICT_DTYPE)
    cnt = _Counters(counters)
    pool = snap["pool"].ctypes.data if snap["pool"] is not None else None
    load().emu_classify(snap["blob"].ctypes.data, snap["hdr"].ctypes.data, pool, snap["jhdr"], None, C.byref(soa), n,
                        out.ctypes.data, None, cnt.ptr)
    cnt.publish()
    return out.reshape(n, 2)


def trace(clf: "gpc.Classifier", pkt):
    """Emulated gpc_trace of one packet (dict of column values): (verdicts (2,), [step dicts])."""
    blob, nw, hdr, _ = clf.debug_image()
    pool, _, jhdr = clf.debug_epoch()
    cols = {k: np.array([v], dtype=gpc.PKT_COLUMNS[k]) for k, v in pkt.items()}
    soa, keep, n = gpc.pkt_soa_host(cols)
    out = np.zeros(2, dtype=gpc.VERDICT_DTYPE)
    steps = (gpc.gpc_trace_step * 8)()
    ns = C.c_uint32()
    load().emu_trace(blob, hdr, pool, jhdr, C.byref(soa), out.ctypes.data, steps, C.byref(ns))
    names = ("table", "verdict", "flags", "conj_id", "priority", "candidates")
    return out, [{k: getattr(steps[i], k) for k in names} for i in range(ns.value)]
