"""ctypes front-end of oracle/ovs_cls.c (TEST INFRASTRUCTURE ONLY): flow text -> C classifier."""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

import numpy as np

from . import cbuild
from .flowtext import parse_flow

NF = 18
F = {"dl_type": 0, "nw_proto": 1, "nw_src": 2, "nw_dst": 3, "ct_nw_src": 4, "ct_nw_dst": 5, "in_port": 6, "reg0": 7,
     "reg1": 8, "reg3": 9, "reg7": 10, "tun_id": 11, "tp_src": 12, "tp_dst": 13, "icmp_type": 12, "icmp_code": 13,
     "ct_state": 14, "conj_id": 15}
TABLE_IDS = {"AntreaPolicyEgressRule": 1, "EgressRule": 2, "EgressDefaultRule": 3, "AntreaPolicyIngressRule": 4,
             "IngressRule": 5, "IngressDefaultRule": 6, "EgressMetric": 7, "IngressMetric": 8, "L3Forwarding": 9,
             "ConntrackCommit": 10, "Output": 11}
A_CONJ, A_SET_REG, A_CT_COMMIT, A_GOTO, A_GROUP = 1, 2, 3, 4, 5


class OFlow(C.Structure):
    _fields_ = [("table", C.c_int32), ("priority", C.c_uint32), ("val", C.c_uint32 * NF), ("mask", C.c_uint32 * NF),
                ("act_off", C.c_int32), ("n_act", C.c_int32), ("soft", C.c_int32)]


class OAction(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("reg", C.c_uint8), ("a", C.c_uint32), ("b", C.c_uint32), ("c", C.c_uint32),
                ("lv", C.c_uint64), ("lm", C.c_uint64)]


class OPkts(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("src", "dst", "sport", "dport", "proto", "out_port", "in_port", "svc_group",
                                          "tun_id", "ct_src", "ct_dst", "ct_state", "dest", "len")]


_lib = None


def load():
    global _lib
    if _lib is None:
        _lib = C.CDLL(cbuild.build())
        _lib.ocls_create.restype = C.c_void_p
        _lib.ocls_create.argtypes = [C.POINTER(OFlow), C.c_int, C.POINTER(OAction), C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_int]
        _lib.ocls_destroy.argtypes = [C.c_void_p]
        _lib.ocls_classify.argtypes = [C.c_void_p, C.POINTER(OPkts), C.c_size_t, C.c_void_p, C.c_int, C.c_int]
        _lib.ocls_counters.restype = C.POINTER(C.c_uint64)
        _lib.ocls_counters.argtypes = [C.c_void_p]
    return _lib


def _convert(flow_lines: List[str]):
    flows, acts, parsed = [], [], []
    for line in flow_lines:
        f = parse_flow(line)
        t = TABLE_IDS.get(f["table"], 0)
        if not (1 <= t <= 8):
            continue
        m = f["match"]
        if any(k.startswith("ipv6") or k.startswith("ct_ipv6") for k in m) or m.get("dl_type", (0x800, 0))[0] != 0x800:
            continue  # never matches the IPv4 packets this checker classifies
        of = OFlow()
        of.table = t
        of.priority = f["priority"]
        ok = True
        for k, (v, mk) in m.items():
            if k == "ct_label":
                full = (1 << 64) - 1 if mk is None else mk
                of.val[16], of.mask[16] = v & 0xFFFFFFFF, full & 0xFFFFFFFF
                of.val[17], of.mask[17] = (v >> 32) & 0xFFFFFFFF, (full >> 32) & 0xFFFFFFFF
                continue
            if k not in F:
                ok = False
                break
            i = F[k]
            if mk is None:
                mk = 0xFFFFFFFF
            if k == "tun_id" and v > 0xFFFFFFFF:
                ok = False
                break
            of.val[i] = v & mk & 0xFFFFFFFF
            of.mask[i] = mk & 0xFFFFFFFF
        if not ok:
            continue
        of.act_off = len(acts)
        soft = bool(f["actions"])
        for a in f["actions"]:
            oa = OAction()
            if a[0] == "conjunction":
                oa.kind, oa.a, oa.b, oa.c = A_CONJ, a[1], a[2], a[3]
            else:
                soft = False
                if a[0] == "set_reg":
                    oa.kind, oa.reg, oa.a, oa.b = A_SET_REG, a[1], a[2], 0xFFFFFFFF if a[3] is None else a[3]
                elif a[0] == "ct_commit":
                    oa.kind, oa.a = A_CT_COMMIT, TABLE_IDS.get(a[1], 0)
                    if a[2]:
                        oa.lv, oa.lm = a[2][0]
                elif a[0] == "goto_table":
                    oa.kind, oa.a = A_GOTO, TABLE_IDS.get(a[1], 0)
                elif a[0] == "group":
                    oa.kind, oa.a = A_GROUP, a[1]
                else:
                    continue
            acts.append(oa)
        of.n_act = len(acts) - of.act_off
        of.soft = int(soft)
        flows.append(of)
    return flows, acts


class CPipeline:
    def __init__(self, flow_lines: List[str], tiers: Optional[Dict[int, int]] = None):
        lib = load()
        flows, acts = _convert(flow_lines)
        self._flows = (OFlow * max(1, len(flows)))(*flows)
        self._acts = (OAction * max(1, len(acts)))(*acts)
        tiers = tiers or {}
        keys = np.array(sorted(tiers), dtype=np.uint32)
        vals = np.array([max(0, min(255, tiers[int(k)])) for k in keys], dtype=np.uint8)
        self._tk, self._tv = keys, vals
        self.n_flows = len(flows)
        self.h = lib.ocls_create(self._flows, len(flows), self._acts, len(acts), keys.ctypes.data, vals.ctypes.data,
                                 len(keys))
        self.flow_meta = flows

    def __del__(self):
        try:
            load().ocls_destroy(self.h)
        except Exception:
            pass

    def classify(self, cols: Dict[str, np.ndarray], threads=1, count=False) -> np.ndarray:
        p = OPkts()
        keep = []
        n = None
        dts = {"src": np.uint32, "dst": np.uint32, "sport": np.uint16, "dport": np.uint16, "proto": np.uint8,
               "out_port": np.uint32, "in_port": np.uint32, "svc_group": np.uint32, "tun_id": np.uint32,
               "ct_src": np.uint32, "ct_dst": np.uint32, "ct_state": np.uint8, "dest": np.uint8, "len": np.uint16}
        for k, dt in dts.items():
            if k in cols:
                a = np.ascontiguousarray(cols[k], dtype=dt)
                keep.append(a)
                setattr(p, k, a.ctypes.data)
                n = len(a)
        out = np.zeros(4 * n, dtype=np.uint32)
        load().ocls_classify(self.h, C.byref(p), n, out.ctypes.data, threads, int(count))
        return out.view(np.dtype([("conj_id", "<u4"), ("action", "u1"), ("table", "u1"), ("tier", "u1"),
                                  ("flags", "u1")])).reshape(n, 2)
