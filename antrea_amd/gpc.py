"""ctypes binding of include/gpc.h (test-harness / bench plumbing).

The product is the C-ABI library `antrea_amd/_build/libgpc.so` (C++ compiler + HIP kernels). This
module only marshals the JSON-style rule records used by the test vectors into `gpc_rule` structs
and numpy packet columns into `gpc_pkt_soa`. It has no classification logic of its own: when no
HIP device is usable every classify call fails with GPC_EDEV.
"""
from __future__ import annotations

import ctypes as C
import ipaddress
import re
import socket
import os
from typing import Dict, List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPC_LIB") or os.path.join(HERE, "_build", "libgpc.so")  # GPC_LIB: experiment builds

GPC_EINVAL, GPC_ENOTFOUND, GPC_ENOCLAUSE, GPC_EDEV, GPC_ERANGE = 2, 1, 5, 4, 7

TABLES = {"AntreaPolicyEgressRule": 1, "EgressRule": 2, "EgressDefaultRule": 3,
          "AntreaPolicyIngressRule": 4, "IngressRule": 5, "IngressDefaultRule": 6}
POLICY_TYPES = {"K8sNetworkPolicy": 0, "AntreaNetworkPolicy": 1, "AntreaClusterNetworkPolicy": 2,
                "AdminNetworkPolicy": 3, "BaselineAdminNetworkPolicy": 4}
RULE_ACTIONS = {None: 0, "Allow": 0, "Drop": 1, "Reject": 2, "Pass": 3}
PROTOCOLS = {None: 0, "TCP": 1, "UDP": 2, "SCTP": 3, "ICMP": 4, "IGMP": 5}
ADDR_KINDS = {"ip": 1, "ipnet": 2, "ofport": 3, "svcgroup": 4, "ctip": 5, "ctipnet": 6, "labelid": 7}
ACT_NAMES = ["NONE", "NO_MATCH", "ALLOW", "DROP", "REJECT", "ISOLATION_DROP", "BYPASS"]

# verdict dtype: gpc_verdict (8 B)
VERDICT_DTYPE = np.dtype([("conj_id", "<u4"), ("action", "u1"), ("table", "u1"), ("tier", "u1"), ("flags", "u1")])
GROUP_KEY_AUTO, GROUP_KEY_ADDR, GROUP_KEY_SCAN = 0, 1, 2  # gpc_group_key

LB_DTYPE = np.dtype([("endpoint_ip", "<u4"), ("endpoint_port", "<u2"), ("flags", "u1"), ("reserved", "u1"),
                     ("group_id", "<u4"), ("out_port", "<u4")])
LB_HIT, LB_NO_ENDPOINT, LB_DNAT, LB_REMOTE = 1, 2, 4, 8
VFLAG_PASS, VFLAG_TIE, VFLAG_PACKETIN = 1, 2, 4  # gpc_verdict.flags
VTABLE_ENDPOINT_DNAT = 4


class gpc_config(C.Structure):
    _fields_ = [("ipv4_enabled", C.c_int32), ("ipv6_enabled", C.c_int32), ("enable_antrea_policy", C.c_int32),
                ("enable_deny_tracking", C.c_int32), ("cookie", C.c_uint64), ("device", C.c_int32),
                ("compact_after", C.c_int32), ("ovs_meters", C.c_int32), ("external_node", C.c_int32),
                ("group_packets", C.c_int32), ("group_key", C.c_int32), ("launch_pacing", C.c_int32),
                ("reserved", C.c_int32 * 1)]


class gpc_addr(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("family", C.c_uint8), ("prefix_len", C.c_uint8), ("reserved", C.c_uint8),
                ("value", C.c_uint32), ("ip", C.c_uint8 * 16)]


class gpc_service(C.Structure):
    _fields_ = [("protocol", C.c_uint8), ("has_port", C.c_uint8), ("has_end_port", C.c_uint8),
                ("has_src_port", C.c_uint8), ("has_src_end_port", C.c_uint8), ("has_icmp_type", C.c_uint8),
                ("has_icmp_code", C.c_uint8), ("has_igmp_type", C.c_uint8), ("port", C.c_uint16),
                ("end_port", C.c_uint16), ("src_port", C.c_uint16), ("src_end_port", C.c_uint16),
                ("icmp_type", C.c_int32), ("icmp_code", C.c_int32), ("igmp_type", C.c_int32),
                ("has_group_address", C.c_uint8), ("group_address", C.c_uint8 * 4), ("reserved", C.c_uint8 * 3)]


class gpc_rule(C.Structure):
    _fields_ = [("direction", C.c_uint8), ("table", C.c_uint8), ("action", C.c_uint8), ("policy_type", C.c_uint8),
                ("has_priority", C.c_uint8), ("enable_logging", C.c_uint8), ("priority", C.c_uint16),
                ("flow_id", C.c_uint32), ("tier_priority", C.c_int32), ("n_from", C.c_int32), ("n_to", C.c_int32),
                ("n_service", C.c_int32), ("from_", C.POINTER(gpc_addr)), ("to", C.POINTER(gpc_addr)),
                ("service", C.POINTER(gpc_service)), ("name", C.c_char_p), ("log_label", C.c_char_p),
                ("policy_namespace", C.c_char_p), ("policy_name", C.c_char_p), ("policy_uid", C.c_char_p)]


class gpc_pkt_soa(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("src", "dst", "sport", "dport", "proto", "out_port", "in_port", "svc_group",
                                          "tun_id", "ct_src", "ct_dst", "ct_state", "dest", "len",
                                          "src6", "dst6", "ct_src6", "ct_dst6", "ct_mark")]


class gpc_trace_step(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("table", "verdict", "flags", "conj_id", "priority", "candidates")]


class gpc_policy_info(C.Structure):
    _fields_ = [("found", C.c_int32), ("policy_type", C.c_uint8), ("of_priority", C.c_uint16),
                ("policy_namespace", C.c_char * 64), ("policy_name", C.c_char * 128), ("policy_uid", C.c_char * 64),
                ("rule_name", C.c_char * 128), ("log_label", C.c_char * 64)]


class gpc_rule_metric(C.Structure):
    _fields_ = [("conj_id", C.c_uint32), ("reserved", C.c_uint32), ("packets", C.c_uint64), ("bytes", C.c_uint64),
                ("sessions", C.c_uint64)]


class gpc_launch_time(C.Structure):
    _fields_ = [("kernel", C.c_char * 32), ("launches", C.c_uint32), ("dropped", C.c_uint32), ("total_ms", C.c_double)]


class gpc_image_stats(C.Structure):
    _fields_ = [("epoch", C.c_uint64), ("device_bytes", C.c_uint64), ("n_rules", C.c_uint32 * 6),
                ("n_hard", C.c_uint32 * 6), ("n_flows", C.c_uint32), ("n_counter_slots", C.c_uint32),
                ("bytes_records", C.c_uint64), ("bytes_ext", C.c_uint64), ("bytes_bucket_offsets", C.c_uint64),
                ("bytes_entries", C.c_uint64), ("bytes_hash", C.c_uint64), ("overlay_bytes", C.c_uint64),
                ("n_overlay_rules", C.c_uint32), ("n_tombstones", C.c_uint32), ("n_full_builds", C.c_uint64),
                ("n_delta_builds", C.c_uint64), ("n_background_builds", C.c_uint64), ("group_key", C.c_uint32),
                ("lane_sort", C.c_uint32), ("v6_full_builds", C.c_uint64), ("v6_delta_builds", C.c_uint64),
                ("v6_overlay_rules", C.c_uint32), ("v6_prefixes", C.c_uint32), ("n_ext_rules", C.c_uint32),
                ("n_ext_values", C.c_uint32), ("n_pool_collections", C.c_uint64)]


class gpc_endpoint(C.Structure):
    _fields_ = [("family", C.c_uint8), ("is_local", C.c_uint8), ("has_node_name", C.c_uint8), ("is_node_ip", C.c_uint8),
                ("port", C.c_uint16), ("reserved", C.c_uint16), ("ip", C.c_uint8 * 16)]


class gpc_service_config(C.Structure):
    _fields_ = [("family", C.c_uint8), ("protocol", C.c_uint8), ("port", C.c_uint16), ("cluster_group_id", C.c_uint32),
                ("local_group_id", C.c_uint32), ("traffic_policy_local", C.c_uint8), ("is_external", C.c_uint8),
                ("is_nodeport", C.c_uint8), ("is_nested", C.c_uint8), ("is_dsr", C.c_uint8), ("reserved", C.c_uint8),
                ("affinity_timeout", C.c_uint16), ("ip", C.c_uint8 * 16)]


EXPORTS = ["gpc_create", "gpc_destroy", "gpc_initialize", "gpc_install_rule", "gpc_batch_install",
           "gpc_uninstall_rule", "gpc_add_rule_addrs", "gpc_del_rule_addrs", "gpc_reassign_priorities",
           "gpc_get_policy_info", "gpc_metrics", "gpc_commit", "gpc_compact", "gpc_classify", "gpc_classify_host", "gpc_counters",
           "gpc_reset_counters", "gpc_dump_flows", "gpc_get_image_stats", "gpc_debug_image", "gpc_debug_epoch", "gpc_load_flows", "gpc_strerror",
           "gpc_install_service_group", "gpc_uninstall_service_group", "gpc_install_endpoint_flows",
           "gpc_uninstall_endpoint_flows", "gpc_install_service_flows", "gpc_uninstall_service_flows", "gpc_install_pod",
           "gpc_uninstall_pod", "gpc_dump_groups", "gpc_classify_lb", "gpc_classify_host_lb", "gpc_debug_service_image",
           "gpc_abi_version", "gpc_set_node_port_addresses", "gpc_classify6", "gpc_classify6_host", "gpc_debug_image6", "gpc_new_dns_conjunction",
           "gpc_add_dns_conj_addrs", "gpc_del_dns_conj_addrs", "gpc_network_policy_flow_keys", "gpc_stream_epoch", "gpc_trace", "gpc_replay",
           "gpc_set_launch_timing", "gpc_launch_times", "gpc_create_multi", "gpc_n_devices", "gpc_classify_on",
           "gpc_classify6_on", "gpc_classify_host_on", "gpc_counters_on", "gpc_debug_epoch6", "gpc_debug_fail_uploads"]

_lib = None


def load(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("libgpc.so not built (run `python -m antrea_amd.build`): %s" % path)
    lib = C.CDLL(path)
    vp, i32, sz = C.c_void_p, C.c_int32, C.c_size_t
    lib.gpc_create.argtypes = [C.POINTER(gpc_config), C.POINTER(vp)]
    lib.gpc_create_multi.argtypes = [C.POINTER(gpc_config), C.POINTER(i32), sz, C.POINTER(vp)]
    lib.gpc_n_devices.argtypes = [vp]
    lib.gpc_classify_on.argtypes = [vp, C.c_uint32, C.POINTER(gpc_pkt_soa), sz, vp, vp, i32, vp]
    lib.gpc_classify6_on.argtypes = [vp, C.c_uint32, C.POINTER(gpc_pkt_soa), sz, vp, i32, vp]
    lib.gpc_classify_host_on.argtypes = [vp, C.c_uint32, C.POINTER(gpc_pkt_soa), sz, vp, vp, i32]
    lib.gpc_counters_on.argtypes = [vp, C.c_uint32, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)),
                                    C.POINTER(sz)]
    lib.gpc_destroy.argtypes = [vp]
    lib.gpc_debug_fail_uploads.argtypes = [vp, C.c_int]
    lib.gpc_destroy.restype = None
    lib.gpc_initialize.argtypes = [vp]
    lib.gpc_install_rule.argtypes = [vp, C.POINTER(gpc_rule)]
    lib.gpc_batch_install.argtypes = [vp, C.POINTER(gpc_rule), sz]
    lib.gpc_uninstall_rule.argtypes = [vp, C.c_uint32, C.POINTER(C.c_uint16), sz, C.POINTER(sz)]
    lib.gpc_add_rule_addrs.argtypes = [vp, C.c_uint32, i32, C.POINTER(gpc_addr), sz, C.POINTER(C.c_uint16), i32, i32]
    lib.gpc_del_rule_addrs.argtypes = [vp, C.c_uint32, i32, C.POINTER(gpc_addr), sz, C.POINTER(C.c_uint16)]
    lib.gpc_reassign_priorities.argtypes = [vp, C.POINTER(C.c_uint16), C.POINTER(C.c_uint16), sz, C.c_uint8]
    lib.gpc_get_policy_info.argtypes = [vp, C.c_uint32, C.POINTER(gpc_policy_info)]
    lib.gpc_metrics.argtypes = [vp, C.POINTER(gpc_rule_metric), sz, C.POINTER(sz)]
    lib.gpc_commit.argtypes = [vp]
    lib.gpc_compact.argtypes = [vp]
    lib.gpc_replay.argtypes = [vp]
    lib.gpc_classify.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, i32, vp]
    lib.gpc_classify_host.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, i32]
    lib.gpc_counters.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz)]
    lib.gpc_reset_counters.argtypes = [vp]
    lib.gpc_dump_flows.argtypes = [vp, C.c_char_p, sz, C.POINTER(sz)]
    lib.gpc_get_image_stats.argtypes = [vp, C.POINTER(gpc_image_stats)]
    lib.gpc_debug_image.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz), C.POINTER(vp), C.POINTER(sz)]
    lib.gpc_debug_epoch.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz), C.POINTER(C.c_uint32)]
    lib.gpc_debug_epoch6.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz), C.POINTER(C.c_uint32)]
    lib.gpc_load_flows.argtypes = [vp, C.c_char_p, sz, i32, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz)]
    u8p = C.POINTER(C.c_uint8)
    lib.gpc_install_service_group.argtypes = [vp, C.c_uint32, i32, C.POINTER(gpc_endpoint), sz]
    lib.gpc_uninstall_service_group.argtypes = [vp, C.c_uint32]
    lib.gpc_install_endpoint_flows.argtypes = [vp, C.c_uint8, C.c_uint8, C.POINTER(gpc_endpoint), sz]
    lib.gpc_uninstall_endpoint_flows.argtypes = [vp, C.c_uint8, C.c_uint8, C.POINTER(gpc_endpoint), sz]
    lib.gpc_install_service_flows.argtypes = [vp, C.POINTER(gpc_service_config)]
    lib.gpc_uninstall_service_flows.argtypes = [vp, u8p, C.c_uint8, C.c_uint16, C.c_uint8]
    lib.gpc_install_pod.argtypes = [vp, u8p, C.c_uint8, C.c_uint32]
    lib.gpc_set_node_port_addresses.argtypes = [vp, u8p, C.c_uint8, sz]
    lib.gpc_uninstall_pod.argtypes = [vp, u8p, C.c_uint8]
    lib.gpc_dump_groups.argtypes = [vp, C.c_char_p, sz, C.POINTER(sz)]
    lib.gpc_classify_lb.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, vp, i32, vp]
    lib.gpc_classify_host_lb.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, vp, i32]
    lib.gpc_debug_service_image.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz)]
    lib.gpc_classify6.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, i32, vp]
    lib.gpc_classify6_host.argtypes = [vp, C.POINTER(gpc_pkt_soa), sz, vp, i32]
    lib.gpc_debug_image6.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(sz), C.POINTER(vp), C.POINTER(sz)]
    lib.gpc_new_dns_conjunction.argtypes = [vp, C.c_uint32]
    lib.gpc_add_dns_conj_addrs.argtypes = [vp, C.c_uint32, C.POINTER(gpc_addr), sz]
    lib.gpc_del_dns_conj_addrs.argtypes = [vp, C.c_uint32, C.POINTER(gpc_addr), sz]
    lib.gpc_network_policy_flow_keys.argtypes = [vp, C.c_char_p, C.c_char_p, C.c_uint8, C.c_char_p, sz, C.POINTER(sz),
                                                 C.POINTER(sz)]
    lib.gpc_stream_epoch.argtypes = [vp, vp, C.POINTER(C.c_uint64)]
    lib.gpc_trace.argtypes = [vp, C.POINTER(gpc_pkt_soa), vp, vp, C.POINTER(gpc_trace_step), sz, C.POINTER(sz)]
    lib.gpc_set_launch_timing.argtypes = [vp, C.c_uint32]
    lib.gpc_launch_times.argtypes = [vp, C.POINTER(gpc_launch_time), sz, C.POINTER(sz)]
    lib.gpc_strerror.argtypes = [i32]
    lib.gpc_strerror.restype = C.c_char_p
    _lib = lib
    return lib


class GpcError(RuntimeError):
    def __init__(self, code, what):
        self.code = -code if code < 0 else code
        super().__init__("%s: %s (%d)" % (what, load().gpc_strerror(code).decode(), code))


def _check(rc, what):
    if rc != 0:
        raise GpcError(rc, what)


# ------------------------------------------------------------------------------ marshalling
_ADDR_NP = np.dtype([("kind", "u1"), ("family", "u1"), ("prefix_len", "u1"), ("reserved", "u1"), ("value", "<u4"),
                     ("ip", "u1", 16)])  # gpc_addr


def _addr(a) -> gpc_addr:
    out = gpc_addr()
    if isinstance(a, str):
        if "." not in a and ":" not in a:
            a = {"ofport": int(a)}
        elif "/" in a:
            a = {"ipnet": a}
        else:
            a = {"ip": a}
    (kind, v), = a.items()
    out.kind = ADDR_KINDS[kind]
    if kind in ("ip", "ctip"):
        ip = ipaddress.ip_address(v)
        out.family = ip.version
        out.ip[:len(ip.packed)] = list(ip.packed)
    elif kind in ("ipnet", "ctipnet"):
        n = ipaddress.ip_network(v, strict=False)
        out.family = n.version
        out.prefix_len = n.prefixlen
        out.ip[:len(n.network_address.packed)] = list(n.network_address.packed)
    else:
        out.value = int(v)
    return out


def _service(s: dict) -> gpc_service:
    out = gpc_service()
    out.protocol = PROTOCOLS[s.get("protocol")]
    for f in ("port", "end_port", "src_port", "src_end_port"):
        if s.get(f) is not None:
            setattr(out, "has_" + f, 1)
            setattr(out, f, int(s[f]))
    for f in ("icmp_type", "icmp_code", "igmp_type"):
        if s.get(f) is not None:
            setattr(out, "has_" + f, 1)
            setattr(out, f, int(s[f]))
    if s.get("group_address"):
        out.has_group_address = 1
        out.group_address[:] = list(ipaddress.ip_address(s["group_address"]).packed)
    return out


def _ip_bytes(ip):
    a = ipaddress.ip_address(ip)
    buf = (C.c_uint8 * 16)()
    buf[:len(a.packed)] = list(a.packed)
    return a.version, buf


def _endpoints(eps):
    """proxy.Endpoint dicts: {"ip", "port", "is_local", "node_name", "is_node_ip"}."""
    arr = (gpc_endpoint * max(1, len(eps)))()
    for i, e in enumerate(eps):
        fam, b = _ip_bytes(e["ip"])
        arr[i].family = fam
        arr[i].ip[:] = list(b)
        arr[i].port = int(e["port"])
        arr[i].is_local = int(bool(e.get("is_local")))
        arr[i].has_node_name = int(bool(e.get("node_name")))
        arr[i].is_node_ip = int(bool(e.get("is_node_ip")))
    return arr


SVC_PROTOCOLS = {"TCP": 1, "UDP": 2, "SCTP": 3}


_OCTET = r"(?:25[0-5]|2[0-4][0-9]|1[0-9][0-9]|[1-9]?[0-9])"
_DOTTED_QUAD = re.compile(r"%s(?:\.%s){3}\Z" % (_OCTET, _OCTET))


class RuleBuf:
    """Keeps the ctypes objects of one or more gpc_rule alive."""

    def __init__(self, rules: List[dict]):
        self.keep = []
        self.arr = (gpc_rule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            self._fill(self.arr[i], r)
        self.n = len(rules)

    def _addrs(self, lst):
        if lst is None:
            return -1, None
        n = len(lst)
        if n >= 64 and all(type(a) is str and _DOTTED_QUAD.match(a) for a in lst):
            # large lists of IPv4 Pod addresses (AddressGroups): filled as one numpy record array
            # in gpc_addr's layout, the dotted quads parsed by inet_aton (C) instead of ipaddress;
            # only plain decimal quads take this path (inet_aton also takes octal / hex / short
            # forms that ipaddress rejects, and IPv4-embedded IPv6 text has colons)
            buf = np.zeros(n, dtype=_ADDR_NP)
            buf["kind"] = ADDR_KINDS["ip"]
            buf["family"] = 4
            buf["ip"][:, :4] = np.frombuffer(b"".join(socket.inet_aton(a) for a in lst), np.uint8).reshape(n, 4)
            self.keep.append(buf)
            return n, (gpc_addr * n).from_buffer(buf)
        arr = (gpc_addr * max(1, n))(*[_addr(a) for a in lst])
        self.keep.append(arr)
        return n, arr

    def _fill(self, g: gpc_rule, r: dict):
        g.direction = 1 if r["direction"] == "Out" else 0
        g.table = TABLES[r["table"]]
        g.action = RULE_ACTIONS[r.get("action")]
        g.policy_type = POLICY_TYPES[r.get("policy_type", "K8sNetworkPolicy")]
        if r.get("priority") is not None:
            g.has_priority = 1
            g.priority = int(r["priority"])
        g.enable_logging = 1 if r.get("enable_logging") else 0
        g.flow_id = int(r["flow_id"])
        g.tier_priority = int(r.get("tier_priority") or 0)
        g.n_from, g.from_ = self._addrs(r.get("from"))
        g.n_to, g.to = self._addrs(r.get("to"))
        svc = r.get("service")
        if svc is None:
            g.n_service = -1
        else:
            arr = (gpc_service * max(1, len(svc)))(*[_service(s) for s in svc])
            self.keep.append(arr)
            g.n_service, g.service = len(svc), arr
        for f in ("name", "log_label", "policy_namespace", "policy_name", "policy_uid"):
            b = (r.get(f) or "").encode()
            self.keep.append(b)
            setattr(g, f, b)


PKT_COLUMNS = {"src": np.uint32, "dst": np.uint32, "sport": np.uint16, "dport": np.uint16, "proto": np.uint8,
               "out_port": np.uint32, "in_port": np.uint32, "svc_group": np.uint32, "tun_id": np.uint32,
               "ct_src": np.uint32, "ct_dst": np.uint32, "ct_state": np.uint8, "dest": np.uint8, "len": np.uint16,
               # IPv6 batches: (n, 16) uint8, network byte order
               "src6": np.uint8, "dst6": np.uint8, "ct_src6": np.uint8, "ct_dst6": np.uint8, "ct_mark": np.uint8}


def pkt_soa_host(cols: Dict[str, np.ndarray]):
    """numpy columns -> (gpc_pkt_soa, keepalive list)."""
    soa = gpc_pkt_soa()
    keep = []
    n = None
    for name, dt in PKT_COLUMNS.items():
        a = cols.get(name)
        if a is None:
            continue
        a = np.ascontiguousarray(a, dtype=dt)
        if n is None:
            n = len(a)
        elif len(a) != n:
            raise ValueError("column %s has %d rows, expected %d" % (name, len(a), n))
        keep.append(a)
        setattr(soa, name, a.ctypes.data)
    return soa, keep, n or 0


def pkt_soa_device(cols: Dict[str, "object"]):
    """torch device tensors -> gpc_pkt_soa of device pointers."""
    soa = gpc_pkt_soa()
    for name in PKT_COLUMNS:
        t = cols.get(name)
        if t is not None:
            setattr(soa, name, t.data_ptr())
    return soa


class Classifier:
    """One gpc context: one control plane over one GPU (`device`) or several (`devices`, a list of
    HIP ordinals: gpc_create_multi; every commit is published on each of them, the `slot` argument
    of the data-path calls picks one, metrics sum over all)."""

    def __init__(self, ipv4=True, ipv6=False, enable_antrea_policy=True, enable_deny_tracking=False,
                 cookie=0x1020000000000, device=0, compact_after=0, ovs_meters=False, k8s_node=True, group_packets=0,
                 group_key=0, devices=None, launch_pacing=0):
        self.lib = load()
        cfg = gpc_config(ipv4_enabled=int(ipv4), ipv6_enabled=int(ipv6),
                         enable_antrea_policy=int(enable_antrea_policy),
                         enable_deny_tracking=int(enable_deny_tracking), cookie=cookie, device=device,
                         compact_after=int(compact_after), ovs_meters=int(ovs_meters),
                         external_node=int(not k8s_node), group_packets=int(group_packets),
                         group_key=int(group_key), launch_pacing=int(launch_pacing))
        h = C.c_void_p()
        if devices is None:
            _check(self.lib.gpc_create(C.byref(cfg), C.byref(h)), "gpc_create")
        else:
            devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            _check(self.lib.gpc_create_multi(C.byref(cfg), devs, len(devices), C.byref(h)), "gpc_create_multi")
        self.h = h

    @property
    def n_devices(self) -> int:
        n = self.lib.gpc_n_devices(self.h)
        _check(min(n, 0), "gpc_n_devices")
        return n

    def close(self):
        if self.h:
            self.lib.gpc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- openflow.Client NP surface
    def initialize(self):
        _check(self.lib.gpc_initialize(self.h), "Initialize")

    def install_policy_rule_flows(self, rule: dict):
        b = RuleBuf([rule])
        _check(self.lib.gpc_install_rule(self.h, b.arr), "InstallPolicyRuleFlows")

    def batch_install_policy_rule_flows(self, rules: List[dict]):
        b = RuleBuf(rules)
        _check(self.lib.gpc_batch_install(self.h, b.arr, b.n), "BatchInstallPolicyRuleFlows")

    def uninstall_policy_rule_flows(self, rule_id: int) -> List[str]:
        st = (C.c_uint16 * 64)()
        n = C.c_size_t()
        _check(self.lib.gpc_uninstall_rule(self.h, rule_id, st, 64, C.byref(n)), "UninstallPolicyRuleFlows")
        return [str(st[i]) for i in range(n.value)]

    def _addr_call(self, fn, rule_id, addr_type, addrs, priority, *extra):
        arr = (gpc_addr * max(1, len(addrs)))(*[_addr(a) for a in addrs])
        p = C.pointer(C.c_uint16(priority)) if priority is not None else None
        return fn(self.h, rule_id, 0 if addr_type == "src" else 1, arr, len(addrs), p, *extra)

    def add_policy_rule_address(self, rule_id, addr_type, addrs, priority=None, enable_logging=False, is_mcnp=False):
        _check(self._addr_call(self.lib.gpc_add_rule_addrs, rule_id, addr_type, addrs, priority,
                               int(enable_logging), int(is_mcnp)), "AddPolicyRuleAddress")

    def delete_policy_rule_address(self, rule_id, addr_type, addrs, priority=None):
        _check(self._addr_call(self.lib.gpc_del_rule_addrs, rule_id, addr_type, addrs, priority),
               "DeletePolicyRuleAddress")

    def rule_addr_ip4(self, add: bool, rule_id: int, addr_type: str, ip4: int, priority=None):
        """AddPolicyRuleAddress (add) / DeletePolicyRuleAddress of one IPv4 host address given as an
        int, through preallocated argument buffers: no string parsing or per-call marshalling, so a
        control loop (bench.py C5) pays the library's cost per op, as a cgo caller would. Not
        thread-safe (one buffer per classifier)."""
        if not hasattr(self, "_fast_addr"):
            self._fast_addr = gpc_addr()
            self._fast_addr.kind = ADDR_KINDS["ip"]
            self._fast_addr.family = 4
            self._fast_prio = C.c_uint16(0)
        a = self._fast_addr
        a.ip[0], a.ip[1], a.ip[2], a.ip[3] = (ip4 >> 24) & 255, (ip4 >> 16) & 255, (ip4 >> 8) & 255, ip4 & 255
        p = None
        if priority is not None:
            self._fast_prio.value = priority
            p = C.pointer(self._fast_prio)
        t = 0 if addr_type == "src" else 1
        if add:
            rc = self.lib.gpc_add_rule_addrs(self.h, rule_id, t, C.byref(a), 1, p, 0, 0)
        else:
            rc = self.lib.gpc_del_rule_addrs(self.h, rule_id, t, C.byref(a), 1, p)
        _check(rc, "AddPolicyRuleAddress" if add else "DeletePolicyRuleAddress")

    def reassign_flow_priorities(self, updates: Dict[int, int], table: str):
        ks = list(updates)
        f = (C.c_uint16 * max(1, len(ks)))(*ks)
        t = (C.c_uint16 * max(1, len(ks)))(*[updates[k] for k in ks])
        _check(self.lib.gpc_reassign_priorities(self.h, f, t, len(ks), TABLES[table]), "ReassignFlowPriorities")

    def get_policy_info_from_conjunction(self, rule_id):
        info = gpc_policy_info()
        _check(self.lib.gpc_get_policy_info(self.h, rule_id, C.byref(info)), "GetPolicyInfoFromConjunction")
        if not info.found:
            return (False, None, "", "", "")
        ref = ({v: k for k, v in POLICY_TYPES.items()}[info.policy_type], info.policy_namespace.decode(),
               info.policy_name.decode(), info.policy_uid.decode())
        return (True, ref, str(info.of_priority), info.rule_name.decode(), info.log_label.decode())

    # --- DNS packet-in conjunction (client.go:310-317)
    def new_dns_packet_in_conjunction(self, conj_id: int):
        _check(self.lib.gpc_new_dns_conjunction(self.h, conj_id), "NewDNSPacketInConjunction")

    def add_address_to_dns_conjunction(self, conj_id: int, addrs):
        arr = (gpc_addr * max(1, len(addrs)))(*[_addr(a) for a in addrs])
        _check(self.lib.gpc_add_dns_conj_addrs(self.h, conj_id, arr, len(addrs)), "AddAddressToDNSConjunction")

    def delete_address_from_dns_conjunction(self, conj_id: int, addrs):
        arr = (gpc_addr * max(1, len(addrs)))(*[_addr(a) for a in addrs])
        _check(self.lib.gpc_del_dns_conj_addrs(self.h, conj_id, arr, len(addrs)), "DeleteAddressFromDNSConjunction")

    def get_network_policy_flow_keys(self, name: str, namespace: str, policy_type: str) -> List[str]:
        need, nk = C.c_size_t(), C.c_size_t()
        args = (self.h, name.encode(), namespace.encode(), POLICY_TYPES[policy_type])
        rc = self.lib.gpc_network_policy_flow_keys(*args, None, 0, C.byref(need), C.byref(nk))
        if rc not in (0, -GPC_ERANGE):
            _check(rc, "GetNetworkPolicyFlowKeys")
        buf = C.create_string_buffer(need.value)
        _check(self.lib.gpc_network_policy_flow_keys(*args, buf, need.value, C.byref(need), C.byref(nk)),
               "GetNetworkPolicyFlowKeys")
        text = buf.value.decode()
        return text.split("\n") if nk.value else []

    def network_policy_metrics(self) -> Dict[int, tuple]:
        n = C.c_size_t()
        _check(self.lib.gpc_metrics(self.h, None, 0, C.byref(n)), "NetworkPolicyMetrics")
        arr = (gpc_rule_metric * max(1, n.value))()
        _check(self.lib.gpc_metrics(self.h, arr, n.value, C.byref(n)), "NetworkPolicyMetrics")
        return {arr[i].conj_id: (arr[i].packets, arr[i].bytes, arr[i].sessions) for i in range(n.value)}

    def load_flows(self, lines, replace=True):
        """Flow-text ingest (ovs-ofctl text, one flow per line). Returns (loaded, skipped)."""
        text = ("\n".join(lines) if not isinstance(lines, (str, bytes)) else lines)
        data = text.encode() if isinstance(text, str) else text
        nl, ns, el = C.c_size_t(), C.c_size_t(), C.c_size_t()
        rc = self.lib.gpc_load_flows(self.h, data, len(data), int(replace), C.byref(nl), C.byref(ns), C.byref(el))
        if rc:
            raise GpcError(rc, "gpc_load_flows (line %d)" % el.value)
        return nl.value, ns.value

    # --- AntreaProxy surface (client.go:710-815)
    def install_service_group(self, group_id, endpoints, with_session_affinity=False):
        _check(self.lib.gpc_install_service_group(self.h, group_id, int(with_session_affinity), _endpoints(endpoints),
                                                  len(endpoints)), "InstallServiceGroup")

    def uninstall_service_group(self, group_id):
        _check(self.lib.gpc_uninstall_service_group(self.h, group_id), "UninstallServiceGroup")

    def install_endpoint_flows(self, protocol, endpoints, family=4):
        _check(self.lib.gpc_install_endpoint_flows(self.h, SVC_PROTOCOLS[protocol], family, _endpoints(endpoints),
                                                   len(endpoints)), "InstallEndpointFlows")

    def uninstall_endpoint_flows(self, protocol, endpoints, family=4):
        _check(self.lib.gpc_uninstall_endpoint_flows(self.h, SVC_PROTOCOLS[protocol], family, _endpoints(endpoints),
                                                     len(endpoints)), "UninstallEndpointFlows")

    def install_service_flows(self, cfg: dict):
        """types.ServiceConfig as a dict: ip, port, protocol, cluster_group_id, local_group_id,
        traffic_policy_local, is_external, is_nodeport, is_nested, is_dsr, affinity_timeout."""
        c = gpc_service_config()
        fam, b = _ip_bytes(cfg["ip"])
        c.family = fam
        c.ip[:] = list(b)
        c.protocol = SVC_PROTOCOLS[cfg["protocol"]]
        c.port = int(cfg["port"])
        c.cluster_group_id = int(cfg.get("cluster_group_id", 0))
        c.local_group_id = int(cfg.get("local_group_id", 0))
        for f in ("traffic_policy_local", "is_external", "is_nodeport", "is_nested", "is_dsr"):
            setattr(c, f, int(bool(cfg.get(f))))
        c.affinity_timeout = int(cfg.get("affinity_timeout", 0))
        _check(self.lib.gpc_install_service_flows(self.h, C.byref(c)), "InstallServiceFlows")

    def uninstall_service_flows(self, ip, port, protocol):
        fam, b = _ip_bytes(ip)
        _check(self.lib.gpc_uninstall_service_flows(self.h, b, fam, int(port), SVC_PROTOCOLS[protocol]),
               "UninstallServiceFlows")

    def install_pod(self, ip, ofport):
        fam, b = _ip_bytes(ip)
        _check(self.lib.gpc_install_pod(self.h, b, fam, int(ofport)), "InstallPodFlows")

    def uninstall_pod(self, ip):
        fam, b = _ip_bytes(ip)
        _check(self.lib.gpc_uninstall_pod(self.h, b, fam), "UninstallPodFlows")

    def set_node_port_addresses(self, ips):
        """NewClient's nodePortAddressesIPv4 with proxyAll (pipeline.go:2282-2314 nodePortMarkFlows);
        [] turns NodePort marking off."""
        buf = (C.c_uint8 * (16 * max(1, len(ips))))()
        for i, ip in enumerate(ips):
            fam, b = _ip_bytes(ip)
            if fam != 4:
                raise GpcError(-GPC_EINVAL, "NodePort addresses: IPv4 only")
            C.memmove(C.byref(buf, 16 * i), b, 4)
        _check(self.lib.gpc_set_node_port_addresses(self.h, buf, 4, len(ips)), "gpc_set_node_port_addresses")

    def dump_groups(self) -> List[str]:
        need = C.c_size_t()
        self.lib.gpc_dump_groups(self.h, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        _check(self.lib.gpc_dump_groups(self.h, buf, need.value, C.byref(need)), "gpc_dump_groups")
        return [l for l in buf.value.decode().split("\n") if l]

    def debug_service_image(self):
        b = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        _check(self.lib.gpc_debug_service_image(self.h, C.byref(b), C.byref(n)), "gpc_debug_service_image")
        return C.cast(b, C.c_void_p).value

    # --- data path
    def commit(self):
        """Publish pending changes (a delta epoch when few rules changed, else a full rebuild)."""
        _check(self.lib.gpc_commit(self.h), "gpc_commit")

    def replay(self):
        """ReplayFlows for the device (gpc_replay): rebuild the device state from the host shadow."""
        _check(self.lib.gpc_replay(self.h), "gpc_replay")

    def compact(self):
        """Publish with a full image rebuild (empties the overlay)."""
        _check(self.lib.gpc_compact(self.h), "gpc_compact")

    def debug_fail_uploads(self, n):
        """Fault injection (tests): the next n device image uploads fail with GPC_EDEV."""
        _check(self.lib.gpc_debug_fail_uploads(self.h, int(n)), "gpc_debug_fail_uploads")

    def classify_host(self, cols: Dict[str, np.ndarray], count=False, lb=False, slot=0):
        """Verdicts (n, 2); with lb=True also the Service stage results (n,) of LB_DTYPE."""
        soa, keep, n = pkt_soa_host(cols)
        out = np.zeros(2 * n, dtype=VERDICT_DTYPE)
        lbo = np.zeros(n, dtype=LB_DTYPE) if lb else None
        _check(self.lib.gpc_classify_host_on(self.h, int(slot), C.byref(soa), n, out.ctypes.data,
                                             lbo.ctypes.data if lb else None, int(count)), "gpc_classify_host")
        return (out.reshape(n, 2), lbo) if lb else out.reshape(n, 2)

    def classify6_host(self, cols: Dict[str, np.ndarray], count=False):
        """IPv6 verdicts (n, 2): cols carries src6 / dst6 as (n, 16) uint8 (network order)."""
        soa, keep, n = pkt_soa_host(cols)
        out = np.zeros(2 * n, dtype=VERDICT_DTYPE)
        _check(self.lib.gpc_classify6_host(self.h, C.byref(soa), n, out.ctypes.data, int(count)), "gpc_classify6_host")
        return out.reshape(n, 2)

    def classify6_device(self, soa: gpc_pkt_soa, n: int, out_ptr: int, count=False, stream: int = 0, slot=0):
        _check(self.lib.gpc_classify6_on(self.h, int(slot), C.byref(soa), n, out_ptr, int(count), stream or None),
               "gpc_classify6")

    def debug_image6(self):
        """(blob pointer, n_words, hdr pointer) of the committed IPv6 image (None when absent)."""
        b = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        h = C.c_void_p()
        hb = C.c_size_t()
        _check(self.lib.gpc_debug_image6(self.h, C.byref(b), C.byref(n), C.byref(h), C.byref(hb)), "gpc_debug_image6")
        return (C.cast(b, C.c_void_p).value if n.value else None), n.value, h.value

    def classify_device(self, soa: gpc_pkt_soa, n: int, out_ptr: int, count=False, stream: int = 0, lb_ptr: int = 0,
                        slot=0):
        _check(self.lib.gpc_classify_on(self.h, int(slot), C.byref(soa), n, out_ptr, lb_ptr or None, int(count),
                                        stream or None), "gpc_classify")

    def trace(self, pkt: Dict[str, int]):
        """gpc_trace of one packet (dict of column values): (verdicts (2,), [step dicts], lb result)."""
        cols = {k: np.array([v], dtype=PKT_COLUMNS[k]) for k, v in pkt.items()}
        soa, keep, n = pkt_soa_host(cols)
        out = np.zeros(2, dtype=VERDICT_DTYPE)
        lb = np.zeros(1, dtype=LB_DTYPE)
        steps = (gpc_trace_step * 8)()
        ns = C.c_size_t()
        _check(self.lib.gpc_trace(self.h, C.byref(soa), out.ctypes.data, lb.ctypes.data, steps, 8, C.byref(ns)),
               "gpc_trace")
        names = ("table", "verdict", "flags", "conj_id", "priority", "candidates")
        return out, [{k: getattr(steps[i], k) for k in names} for i in range(ns.value)], lb[0]

    def stream_epoch(self, stream: int = 0) -> int:
        """Epoch the last classify launch on `stream` was bound to (gpc_stream_epoch)."""
        e = C.c_uint64()
        _check(self.lib.gpc_stream_epoch(self.h, stream or None, C.byref(e)), "gpc_stream_epoch")
        return e.value

    def set_launch_timing(self, slots: int):
        """gpc_set_launch_timing: HIP events around every kernel of the next gpc_classify* calls."""
        _check(self.lib.gpc_set_launch_timing(self.h, int(slots)), "gpc_set_launch_timing")

    def launch_times(self) -> Dict[str, dict]:
        """gpc_launch_times: {kernel: {"launches", "total_ms", "mean_ms", "dropped"}} since the last call."""
        arr = (gpc_launch_time * 8)()
        n = C.c_size_t()
        _check(self.lib.gpc_launch_times(self.h, arr, 8, C.byref(n)), "gpc_launch_times")
        return {arr[i].kernel.decode(): {"launches": arr[i].launches, "total_ms": arr[i].total_ms,
                                         "mean_ms": arr[i].total_ms / max(1, arr[i].launches),
                                         "dropped": arr[i].dropped} for i in range(n.value)}

    def counters(self, slot=0):
        p = C.POINTER(C.c_uint64)()
        s = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        _check(self.lib.gpc_counters_on(self.h, int(slot), C.byref(p), C.byref(s), C.byref(n)), "gpc_counters")
        slots = [s[i] for i in range(n.value)]
        return C.cast(p, C.c_void_p).value, slots

    def reset_counters(self):
        _check(self.lib.gpc_reset_counters(self.h), "gpc_reset_counters")

    # --- introspection
    def dump_flows(self) -> List[str]:
        need = C.c_size_t()
        self.lib.gpc_dump_flows(self.h, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        _check(self.lib.gpc_dump_flows(self.h, buf, need.value, C.byref(need)), "gpc_dump_flows")
        return [l for l in buf.value.decode().split("\n") if l]

    def debug_image(self):
        """(blob pointer, n_words, hdr pointer, hdr_bytes) of the last committed host image."""
        b = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        h = C.c_void_p()
        hb = C.c_size_t()
        _check(self.lib.gpc_debug_image(self.h, C.byref(b), C.byref(n), C.byref(h), C.byref(hb)), "gpc_debug_image")
        return C.cast(b, C.c_void_p).value, n.value, h.value, hb.value

    def debug_epoch(self):
        """(journal pool pointer or None, pool words, JournalHdr offset) of the current epoch's host
        mirror (None / 0 / 0 when the epoch is the base image alone)."""
        p = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        h = C.c_uint32()
        _check(self.lib.gpc_debug_epoch(self.h, C.byref(p), C.byref(n), C.byref(h)), "gpc_debug_epoch")
        return C.cast(p, C.c_void_p).value, n.value, h.value

    def debug_epoch6(self):
        """debug_epoch for the IPv6 image's journal."""
        p = C.POINTER(C.c_uint32)()
        n = C.c_size_t()
        h = C.c_uint32()
        _check(self.lib.gpc_debug_epoch6(self.h, C.byref(p), C.byref(n), C.byref(h)), "gpc_debug_epoch6")
        return C.cast(p, C.c_void_p).value, n.value, h.value

    def image_stats(self) -> dict:
        st = gpc_image_stats()
        _check(self.lib.gpc_get_image_stats(self.h, C.byref(st)), "gpc_get_image_stats")
        return {"epoch": st.epoch, "device_bytes": st.device_bytes, "n_rules": list(st.n_rules),
                "n_hard": list(st.n_hard), "n_flows": st.n_flows, "n_counter_slots": st.n_counter_slots,
                "bytes": {"records": st.bytes_records, "ext": st.bytes_ext, "bucket_offsets": st.bytes_bucket_offsets,
                          "entries": st.bytes_entries, "hash": st.bytes_hash},
                "overlay_bytes": st.overlay_bytes, "n_overlay_rules": st.n_overlay_rules,
                "n_tombstones": st.n_tombstones, "n_full_builds": st.n_full_builds,
                "n_delta_builds": st.n_delta_builds, "n_background_builds": st.n_background_builds,
                "group_key": st.group_key, "lane_sort": [st.lane_sort & 0xff, st.lane_sort >> 8],
                "v6_full_builds": st.v6_full_builds, "v6_delta_builds": st.v6_delta_builds,
                "v6_overlay_rules": st.v6_overlay_rules, "v6_prefixes": st.v6_prefixes,
                "n_ext_rules": st.n_ext_rules, "n_ext_values": st.n_ext_values,
                "n_pool_collections": st.n_pool_collections}
