"""ctypes front-end of oracle/ovs_cls.c (TEST INFRASTRUCTURE ONLY): flow text -> C classifier."""
from __future__ import annotations

import ctypes as C
import os
import zlib
from typing import Dict, List, Optional

import numpy as np

from . import cbuild
from .flowtext import parse_flow

NF = 20
F = {"dl_type": 0, "nw_proto": 1, "nw_src": 2, "nw_dst": 3, "ct_nw_src": 4, "ct_nw_dst": 5, "in_port": 6, "reg0": 7,
     "reg1": 8, "reg3": 9, "reg7": 10, "tun_id": 11, "tp_src": 12, "tp_dst": 13, "icmp_type": 12, "icmp_code": 13,
     "ct_state": 14, "conj_id": 15, "ct_mark": 18, "reg4": 19}
TABLE_IDS = {"AntreaPolicyEgressRule": 1, "EgressRule": 2, "EgressDefaultRule": 3, "AntreaPolicyIngressRule": 4,
             "IngressRule": 5, "IngressDefaultRule": 6, "EgressMetric": 7, "IngressMetric": 8, "L3Forwarding": 9,
             "ConntrackCommit": 10, "Output": 11, "IngressSecurityClassifier": 12, "ServiceLB": 13,
             "EndpointDNAT": 14}
KEEP_TABLES = {1, 2, 3, 4, 5, 6, 7, 8, 12, 13, 14}
A_CONJ, A_SET_REG, A_CT_COMMIT, A_GOTO, A_GROUP, A_CONTROLLER = 1, 2, 3, 4, 5, 6

# numpy twins of the C records (same layout as ocls_flow / ocls_action)
FLOW_DT = np.dtype([("table", "<i4"), ("priority", "<u4"), ("val", "<u4", (NF,)), ("mask", "<u4", (NF,)),
                    ("act_off", "<i4"), ("n_act", "<i4"), ("soft", "<i4"), ("sig", "<u4")])
ACT_DT = np.dtype({"names": ["kind", "reg", "a", "b", "c", "lv", "lm"],
                   "formats": ["u1", "u1", "<u4", "<u4", "<u4", "<u8", "<u8"],
                   "offsets": [0, 1, 4, 8, 12, 16, 24], "itemsize": 32})
STAT_NAMES = ("lookups", "subtables_probed", "subtables_skipped_by_trie", "soft_matches", "soft_levels",
              "conj_actions_hashed")


class OPkts(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("src", "dst", "sport", "dport", "proto", "out_port", "in_port", "svc_group",
                                          "tun_id", "ct_src", "ct_dst", "ct_state", "dest", "len", "ct_mark")]


_lib = None


def load():
    global _lib
    if _lib is None:
        _lib = C.CDLL(cbuild.build())
        _lib.ocls_create.restype = C.c_void_p
        _lib.ocls_create.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        _lib.ocls_destroy.argtypes = [C.c_void_p]
        _lib.ocls_classify.argtypes = [C.c_void_p, C.POINTER(OPkts), C.c_size_t, C.c_void_p, C.c_int, C.c_int]
        _lib.ocls_classify_lb.argtypes = [C.c_void_p, C.POINTER(OPkts), C.c_size_t, C.c_void_p, C.c_void_p, C.c_int,
                                          C.c_int]
        _lib.ocls_set_services.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int]
        _lib.ocls_counters.restype = C.POINTER(C.c_uint64)
        _lib.ocls_counters.argtypes = [C.c_void_p]
        _lib.ocls_stats.argtypes = [C.c_void_p, C.c_void_p]
        _lib.ocls_n_subtables.argtypes = [C.c_void_p, C.c_int]
    return _lib


def _verdict_sig(actions) -> int:
    """Signature of a hard flow's verdict (oracle/ovs_cls.py _verdict_sig): equal-priority
    overlapping hard flows with different signatures are a TIE."""
    acts = [a for a in actions if a[0] in ("drop", "goto_table", "ct_commit", "group")]
    sig = tuple(a[0] + str(a[1] if len(a) > 1 else "") for a in acts) or ("drop",)
    return zlib.crc32(repr(sig).encode())


def _convert_lines(flow_lines: List[str]):
    """Flow text -> (flow records, action records, index of each kept flow in flow_lines)."""
    flows = np.zeros(len(flow_lines), FLOW_DT)
    acts = []
    kept = []
    k = 0
    for li, line in enumerate(flow_lines):
        f = parse_flow(line)
        t = TABLE_IDS.get(f["table"], 0)
        if t not in KEEP_TABLES:
            continue
        m = f["match"]
        if any(x.startswith("ipv6") or x.startswith("ct_ipv6") for x in m) or m.get("dl_type", (0x800, 0))[0] != 0x800:
            continue  # never matches the IPv4 packets this checker classifies
        rec = flows[k]
        ok = True
        for key, (v, mk) in m.items():
            if key == "ct_label":
                full = (1 << 64) - 1 if mk is None else mk
                rec["val"][16], rec["mask"][16] = v & 0xFFFFFFFF, full & 0xFFFFFFFF
                rec["val"][17], rec["mask"][17] = (v >> 32) & 0xFFFFFFFF, (full >> 32) & 0xFFFFFFFF
                continue
            if key not in F:
                ok = False
                break
            i = F[key]
            if mk is None:
                mk = 0xFFFFFFFF
            if key == "tun_id" and v > 0xFFFFFFFF:
                ok = False
                break
            rec["val"][i] = v & mk & 0xFFFFFFFF
            rec["mask"][i] = mk & 0xFFFFFFFF
        if not ok:
            rec["val"][:] = 0
            rec["mask"][:] = 0
            continue
        rec["table"] = t
        rec["priority"] = f["priority"]
        off = len(acts)
        soft = bool(f["actions"])
        for a in f["actions"]:
            if a[0] == "conjunction":
                acts.append((A_CONJ, 0, a[1], a[2], a[3], 0, 0))
                continue
            soft = False
            if a[0] == "set_reg":
                acts.append((A_SET_REG, a[1], a[2] & 0xFFFFFFFF, 0xFFFFFFFF if a[3] is None else a[3], 0, 0, 0))
            elif a[0] == "ct_commit":
                lv, lm = a[2][0] if a[2] else (0, 0)
                nat = a[3] if len(a) > 3 else None  # EndpointDNAT: nat(dst=ip:port)
                acts.append((A_CT_COMMIT, 0, TABLE_IDS.get(a[1], 0), nat[0] if nat else 0,
                             (nat[1] | 0x10000) if nat else 0, lv, lm))
            elif a[0] == "goto_table":
                acts.append((A_GOTO, 0, TABLE_IDS.get(a[1], 0), 0, 0, 0, 0))
            elif a[0] == "group":
                acts.append((A_GROUP, 0, a[1], 0, 0, 0, 0))
            elif a[0] == "controller":
                acts.append((A_CONTROLLER, 0, 0, 0, 0, 0, 0))
        rec["act_off"] = off
        rec["n_act"] = len(acts) - off
        rec["soft"] = int(soft)
        rec["sig"] = 0 if soft else _verdict_sig(f["actions"])
        kept.append(li)
        k += 1
    return flows[:k].copy(), np.array(acts, dtype=ACT_DT) if acts else np.zeros(0, ACT_DT), kept


def _convert_chunk(args):
    lines, base = args
    fl, ac, kept = _convert_lines(lines)
    return fl, ac, [base + i for i in kept]


def _convert(flow_lines: List[str], procs: Optional[int] = None):
    """Parallel conversion of large dumps (a fork pool over chunks; the oracle never touches a GPU)."""
    n = len(flow_lines)
    procs = procs if procs is not None else min(16, os.cpu_count() or 1)
    if n < 50000 or procs <= 1:
        return _convert_lines(flow_lines)
    import multiprocessing as mp
    step = (n + 4 * procs - 1) // (4 * procs)
    chunks = [(flow_lines[i:i + step], i) for i in range(0, n, step)]
    with mp.get_context("fork").Pool(procs) as pool:
        parts = pool.map(_convert_chunk, chunks)
    flows, acts, kept = [], [], []
    off = 0
    for fl, ac, kp in parts:
        fl = fl.copy()
        fl["act_off"] += off
        off += len(ac)
        flows.append(fl)
        acts.append(ac)
        kept.extend(kp)
    # concatenate packs the padded action dtype: restore the C layout
    return np.concatenate(flows).astype(FLOW_DT), np.concatenate(acts).astype(ACT_DT), kept


class CPipeline:
    def __init__(self, flow_lines: List[str], tiers: Optional[Dict[int, int]] = None, procs: Optional[int] = None):
        lib = load()
        flow_lines = list(flow_lines)
        flows, acts, kept = _convert(flow_lines, procs)
        self._flows = np.ascontiguousarray(flows, dtype=FLOW_DT)
        self._acts = np.ascontiguousarray(acts, dtype=ACT_DT)
        assert self._flows.dtype.itemsize == 184 and self._acts.dtype.itemsize == 32
        tiers = tiers or {}
        keys = np.array(sorted(tiers), dtype=np.uint32)
        vals = np.array([max(0, min(255, tiers[int(k)])) for k in keys], dtype=np.uint8)
        self._tk, self._tv = keys, vals
        self.n_flows = len(flows)
        self._metric_lines = [(i, flow_lines[li]) for i, li in enumerate(kept) if flows[i]["table"] in (7, 8)]
        self.h = lib.ocls_create(self._flows.ctypes.data, len(flows), self._acts.ctypes.data, len(acts),
                                 keys.ctypes.data, vals.ctypes.data, len(keys))

    def __del__(self):
        try:
            load().ocls_destroy(self.h)
        except Exception:
            pass

    def set_services(self, group_lines: List[str], pods: Dict[int, int]):
        """The AntreaProxy stage's select groups (ovs-ofctl dump-groups text) and the Pod map
        (IP -> ofport) of L3Forwarding; ServiceLB / EndpointDNAT flows come with the flow text."""
        from .flowtext import parse_group
        words = []
        for line in group_lines:
            g = parse_group(line)
            words += [g["id"], len(g["buckets"])]
            for b in g["buckets"]:
                sets = [a for a in b["actions"] if a[0] == "set_reg"]
                words.append(len(sets))
                for a in sets:
                    words += [a[1], a[2] & 0xFFFFFFFF, 0xFFFFFFFF if a[3] is None else a[3]]
        self._gw = np.array(words, dtype=np.uint32)
        self._pip = np.array(sorted(pods), dtype=np.uint32)
        self._pport = np.array([pods[int(k)] for k in self._pip], dtype=np.uint32)
        rc = load().ocls_set_services(self.h, self._gw.ctypes.data, len(self._gw), self._pip.ctypes.data,
                                      self._pport.ctypes.data, len(self._pip))
        assert rc == 0, "malformed group encoding"

    def classify(self, cols: Dict[str, np.ndarray], threads=1, count=False, lb=False):
        """Verdicts (n, 2); with lb=True also the Service stage's gpc_lb_result words (n, 4)."""
        p = OPkts()
        keep = []
        n = None
        dts = {"src": np.uint32, "dst": np.uint32, "sport": np.uint16, "dport": np.uint16, "proto": np.uint8,
               "out_port": np.uint32, "in_port": np.uint32, "svc_group": np.uint32, "tun_id": np.uint32,
               "ct_src": np.uint32, "ct_dst": np.uint32, "ct_state": np.uint8, "dest": np.uint8, "len": np.uint16,
               "ct_mark": np.uint8}
        for k, dt in dts.items():
            if k in cols:
                a = np.ascontiguousarray(cols[k], dtype=dt)
                keep.append(a)
                setattr(p, k, a.ctypes.data)
                n = len(a)
        out = np.zeros(4 * n, dtype=np.uint32)
        lbo = np.zeros(4 * n, dtype=np.uint32) if lb else None
        load().ocls_classify_lb(self.h, C.byref(p), n, out.ctypes.data, lbo.ctypes.data if lb else None, threads,
                                int(count))
        v = out.view(np.dtype([("conj_id", "<u4"), ("action", "u1"), ("table", "u1"), ("tier", "u1"),
                               ("flags", "u1")])).reshape(n, 2)
        return (v, lbo.reshape(n, 4)) if lb else v

    def stats(self) -> Dict[str, int]:
        out = np.zeros(8, np.uint64)
        load().ocls_stats(self.h, out.ctypes.data)
        return {k: int(v) for k, v in zip(STAT_NAMES, out)}

    def n_subtables(self) -> List[int]:
        return [load().ocls_n_subtables(self.h, t) for t in (1, 2, 3, 4, 5, 6, 7, 8, 12)]

    def metric_dumps(self) -> Dict[str, List[str]]:
        """ovs-ofctl dump of the two Metric tables with the packet / byte counters accumulated by
        classify(count=True), in the text NetworkPolicyMetrics parses (network_policy.go:2034)."""
        cnt = load().ocls_counters(self.h)
        out = {"EgressMetric": [], "IngressMetric": []}
        for i, line in self._metric_lines:
            f = parse_flow(line)
            head, _, acts = line.partition(" actions=")
            toks = [t for t in head.replace(", ", ",").split(",") if t and not t.startswith(("n_packets=", "n_bytes="))]
            toks = [t for t in toks if not t.startswith("table=")]
            out[f["table"]].append("table=%s, n_packets=%d, n_bytes=%d, %s actions=%s" % (
                f["table"], cnt[2 * i], cnt[2 * i + 1], ",".join(toks), acts))
        return out
