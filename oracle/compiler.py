"""Oracle restatement of Antrea's conjunctive-match compiler (TEST INFRASTRUCTURE ONLY).

Restates, function by function, the NetworkPolicy half of `openflow.Client`:

* match keys                         `pkg/agent/openflow/network_policy.go:38-81`
* address match keys / values        `network_policy.go:97-307`
* matchPair.KeyString / global key   `network_policy.go:325-400`
* conjMatchFlowContext life cycle    `network_policy.go:442-646, 791-864, 1049-1126`
* clause / conjunction calculation   `network_policy.go:1186-1228, 1408-1489`
* Install / Batch / Uninstall        `network_policy.go:1160-1183, 1310-1356, 1570-1624`
* Add / Delete rule address          `network_policy.go:1661-1710`
* ReassignFlowPriorities             `network_policy.go:1746-1889`
* GetPolicyInfoFromConjunction       `network_policy.go:1555-1565`
* service match pairs / port ranges  `network_policy.go:891-1017`, `third_party/networkpolicy/port_range.go:45-132`
* flow builders                      `pkg/agent/openflow/pipeline.go:1604-1670, 1718-1886, 1896-2076`
* initFlows (classifier, skip, log)  `network_policy.go:2126-2269`, `pipeline.go:2144-2182`
* DNS packet-in conjunction          `network_policy.go:697-789`, `pipeline.go:2080-2093`
* GetNetworkPolicyFlowKeys           `network_policy.go:1520-1545, 1712-1736`
* flow -> ovs-ofctl text             `pkg/ovs/openflow/utils.go:255-580, 748-752, 905-1241`

Input records are plain dicts (the JSON test-vector format, see tests/golden/README.md), so this
module has no dependency on the product package.
"""
from __future__ import annotations

import ipaddress
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

# ---------------------------------------------------------------------------------------------
# pipeline constants (pipeline.go:150-176, 207-213, 321-331; fields.go:63-163, 224-227)
# ---------------------------------------------------------------------------------------------
PRIORITY_HIGH = 210
PRIORITY_NORMAL = 200
PRIORITY_LOW = 190
PRIORITY_TOP_ANTREA_POLICY = 64990
PRIORITY_DNS_INTERCEPT = 64991
# PacketInTableField (reg2[0..7]) carries the rule table's OpenFlow table ID, which depends on the
# agent's realized pipeline; the restatement (like libgpc, model.hpp TB_*) numbers the six rule
# tables 1-6. The logging-and-resubmit groups take the group IDs initGroups allocates in order
# (network_policy.go:2271-2300, Multicast off): EgressRule 1, EgressMetric 2, IngressRule 3,
# IngressMetric 4 (as in client_test.go:2762-2767).
TABLE_NUM = {"AntreaPolicyEgressRule": 1, "EgressRule": 2, "EgressDefaultRule": 3, "AntreaPolicyIngressRule": 4,
             "IngressRule": 5, "IngressDefaultRule": 6}
LOGGING_GROUP = {"EgressRule": 1, "EgressMetric": 2, "IngressRule": 3, "IngressMetric": 4}
DNS_PORT = 53
PACKET_IN_METER_NP, PACKET_IN_METER_DNS = 256, 258          # client.go:851-858 meter ids
PACKET_IN_CATEGORY_NP, PACKET_IN_CATEGORY_DNS = 1, 2       # packetin.go:44-52
CONTROLLER_ID = 32776                                       # the agent's OpenFlow controller id
# IngressSecurityClassifier marks (fields.go PktDestinationField reg0[4..7], HairpinCTMark ct_mark[6])
TO_GATEWAY, TO_TUNNEL, TO_UPLINK = 0x20, 0x10, 0x40
HAIRPIN_CT_MARK = 0x40

CT_ZONE = 0xFFF0
CT_ZONE_V6 = 0xFFE6
UNKNOWN_LABEL_IDENTITY = 0xFFFFFF  # multicluster.go:33

DISPOSITION_ALLOW, DISPOSITION_DROP, DISPOSITION_REJ, DISPOSITION_PASS = 0, 1, 2, 3

EGRESS_TABLES_ORDER = ["EgressSecurityClassifier", "AntreaPolicyEgressRule", "EgressRule",
                       "EgressDefaultRule", "EgressMetric", "L3Forwarding"]
INGRESS_TABLES_ORDER = ["IngressSecurityClassifier", "AntreaPolicyIngressRule", "IngressRule",
                        "IngressDefaultRule", "IngressMetric", "ConntrackCommit"]
NEXT_TABLE = {}
for _order in (EGRESS_TABLES_ORDER, INGRESS_TABLES_ORDER):
    for _a, _b in zip(_order, _order[1:]):
        NEXT_TABLE[_a] = _b

K8S_NP = "K8sNetworkPolicy"


# ---------------------------------------------------------------------------------------------
# match keys (network_policy.go:38-81)
# ---------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class MatchKey:
    name: str
    proto: str       # binding.Protocol of the key
    category: str    # types.AddressCategory
    key: str         # keyString


def _mk(name, proto, cat, key):
    return MatchKey(name, proto, cat, key)


MatchDstIP = _mk("MatchDstIP", "ip", "IPAddr", "nw_dst")
MatchSrcIP = _mk("MatchSrcIP", "ip", "IPAddr", "nw_src")
MatchDstIPNet = _mk("MatchDstIPNet", "ip", "IPNetAddr", "nw_dst")
MatchSrcIPNet = _mk("MatchSrcIPNet", "ip", "IPNetAddr", "nw_src")
MatchCTDstIP = _mk("MatchCTDstIP", "ip", "IPAddr", "ct_nw_dst")
MatchCTSrcIP = _mk("MatchCTSrcIP", "ip", "IPAddr", "ct_nw_src")
MatchCTDstIPNet = _mk("MatchCTDstIPNet", "ip", "IPNetAddr", "ct_nw_dst")
MatchCTSrcIPNet = _mk("MatchCTSrcIPNet", "ip", "IPNetAddr", "ct_nw_src")
MatchDstIPv6 = _mk("MatchDstIPv6", "ipv6", "IPAddr", "ipv6_dst")
MatchSrcIPv6 = _mk("MatchSrcIPv6", "ipv6", "IPAddr", "ipv6_src")
MatchDstIPNetv6 = _mk("MatchDstIPNetv6", "ipv6", "IPNetAddr", "ipv6_dst")
MatchSrcIPNetv6 = _mk("MatchSrcIPNetv6", "ipv6", "IPNetAddr", "ipv6_src")
MatchCTDstIPv6 = _mk("MatchCTDstIPv6", "ipv6", "IPAddr", "ct_ipv6_dst")
MatchCTSrcIPv6 = _mk("MatchCTSrcIPv6", "ipv6", "IPAddr", "ct_ipv6_src")
MatchCTDstIPNetv6 = _mk("MatchCTDstIPNetv6", "ipv6", "IPNetAddr", "ct_ipv6_dst")
MatchCTSrcIPNetv6 = _mk("MatchCTSrcIPNetv6", "ipv6", "IPNetAddr", "ct_ipv6_src")
MatchDstOFPort = _mk("MatchDstOFPort", "ip", "OFPortAddr", "reg1[0..31]")
MatchSrcOFPort = _mk("MatchSrcOFPort", "ip", "OFPortAddr", "in_port")
MatchTCPDstPort = _mk("MatchTCPDstPort", "tcp", "L4PortAddr", "tp_dst")
MatchTCPv6DstPort = _mk("MatchTCPv6DstPort", "tcp6", "L4PortAddr", "tp_dst")
MatchUDPDstPort = _mk("MatchUDPDstPort", "udp", "L4PortAddr", "tp_dst")
MatchUDPv6DstPort = _mk("MatchUDPv6DstPort", "udp6", "L4PortAddr", "tp_dst")
MatchSCTPDstPort = _mk("MatchSCTPDstPort", "sctp", "L4PortAddr", "tp_dst")
MatchSCTPv6DstPort = _mk("MatchSCTPv6DstPort", "sctp6", "L4PortAddr", "tp_dst")
MatchSCTPSrcPort = _mk("MatchSCTPSrcPort", "sctp", "L4PortAddr", "tp_src")
MatchSCTPv6SrcPort = _mk("MatchSCTPv6SrcPort", "sctp6", "L4PortAddr", "tp_src")
MatchTCPSrcPort = _mk("MatchTCPSrcPort", "tcp", "L4PortAddr", "tp_src")
MatchTCPv6SrcPort = _mk("MatchTCPv6SrcPort", "tcp6", "L4PortAddr", "tp_src")
MatchUDPSrcPort = _mk("MatchUDPSrcPort", "udp", "L4PortAddr", "tp_src")
MatchUDPv6SrcPort = _mk("MatchUDPv6SrcPort", "udp6", "L4PortAddr", "tp_src")
MatchICMPType = _mk("MatchICMPType", "icmp", "ICMPAddr", "icmp_type")
MatchICMPCode = _mk("MatchICMPCode", "icmp", "ICMPAddr", "icmp_code")
MatchICMPv6Type = _mk("MatchICMPv6Type", "icmp6", "ICMPAddr", "icmpv6_type")
MatchICMPv6Code = _mk("MatchICMPv6Code", "icmp6", "ICMPAddr", "icmpv6_code")
MatchServiceGroupID = _mk("MatchServiceGroupID", "ip", "ServiceGroupIDAddr", "reg7[0..31]")
MatchIGMPProtocol = _mk("MatchIGMPProtocol", "igmp", "IGMPAddr", "igmp")
MatchLabelID = _mk("MatchLabelID", "ip", "LabelIDAddr", "tun_id")
MatchCTState = _mk("MatchCTState", "ip", "CTStateAddr", "ct_state")

# The global-map key treats IP and IP/32 (IP/128) as one condition (network_policy.go:341-363).
_IP_KEY_NORMALIZE = {
    MatchDstIP: MatchDstIPNet, MatchDstIPv6: MatchDstIPNetv6,
    MatchSrcIP: MatchSrcIPNet, MatchSrcIPv6: MatchSrcIPNetv6,
}

PROTO_NUM = {"tcp": 6, "udp": 17, "sctp": 132, "icmp": 1, "igmp": 2,
             "tcp6": 6, "udp6": 17, "sctp6": 132, "icmp6": 58}
PROTO_ETH = {"ip": 0x0800, "ipv6": 0x86DD, "tcp": 0x0800, "udp": 0x0800, "sctp": 0x0800,
             "icmp": 0x0800, "igmp": 0x0800, "tcp6": 0x86DD, "udp6": 0x86DD, "sctp6": 0x86DD,
             "icmp6": 0x86DD}


# ---------------------------------------------------------------------------------------------
# addresses (network_policy.go:97-307)
# ---------------------------------------------------------------------------------------------
def parse_address(a):
    """Accepts the test-vector dict form or the compact string form of network_policy_test.go:965."""
    if isinstance(a, str):
        if "." not in a and ":" not in a:
            return ("ofport", int(a))
        if "/" in a:
            return ("ipnet", ipaddress.ip_network(a, strict=False))
        return ("ip", ipaddress.ip_address(a))
    (kind, v), = a.items()
    if kind in ("ip", "ctip"):
        return (kind, ipaddress.ip_address(v))
    if kind in ("ipnet", "ctipnet"):
        return (kind, ipaddress.ip_network(v, strict=False))
    if kind in ("ofport", "svcgroup", "labelid"):
        return (kind, int(v))
    raise ValueError("unknown address kind %r" % (kind,))


def address_match_key(addr, src: bool) -> MatchKey:
    kind, v = addr
    v6 = getattr(v, "version", 4) == 6
    if kind == "ip":
        return (MatchSrcIPv6 if v6 else MatchSrcIP) if src else (MatchDstIPv6 if v6 else MatchDstIP)
    if kind == "ipnet":
        return (MatchSrcIPNetv6 if v6 else MatchSrcIPNet) if src else (MatchDstIPNetv6 if v6 else MatchDstIPNet)
    if kind == "ofport":
        return MatchSrcOFPort if src else MatchDstOFPort
    if kind == "svcgroup":
        return MatchServiceGroupID
    if kind == "ctip":
        return (MatchCTSrcIPv6 if v6 else MatchCTSrcIP) if src else (MatchCTDstIPv6 if v6 else MatchCTDstIP)
    if kind == "ctipnet":
        return (MatchCTSrcIPNetv6 if v6 else MatchCTSrcIPNet) if src else (MatchCTDstIPNetv6 if v6 else MatchCTDstIPNet)
    if kind == "labelid":
        return MatchLabelID
    raise ValueError(kind)


# match values are tagged tuples: ("ip", addr) ("ipnet", net) ("int", n) ("bitrange", v, m|None)
# ("icmp", n|None) ("ctstate", data, mask)
def address_match_value(addr):
    kind, v = addr
    if kind in ("ip", "ctip"):
        return ("ip", v)
    if kind in ("ipnet", "ctipnet"):
        return ("ipnet", v)
    return ("int", v)


def match_pair_key_string(key: MatchKey, value) -> str:
    """matchPair.KeyString (network_policy.go:336-386); only its equivalence classes matter."""
    tag = value[0]
    if tag == "ip":
        ip = value[1]
        vs = "%s/%d" % (ip, 32 if ip.version == 4 else 128)
        key = _IP_KEY_NORMALIZE.get(key, key)
    elif tag == "ipnet":
        vs = str(value[1])
    elif tag == "bitrange":
        vs = "%d/%d" % (value[1], value[2] if value[2] is not None else 65535)
    elif tag == "icmp":
        vs = "%d" % value[1] if value[1] is not None else "<nil>"
    elif tag == "ctstate":
        vs = "%d/%d" % (value[1], value[2])
    else:
        vs = "%d" % value[1]
    return "%s=%s" % (key.name, vs)


# ---------------------------------------------------------------------------------------------
# port ranges (third_party/networkpolicy/port_range.go:45-132)
# ---------------------------------------------------------------------------------------------
def bitwise_match(start: int, end: int) -> List[Tuple[int, int]]:
    if start <= 0 or end <= 0 or start > end:
        raise ValueError("invalid port range")
    if start == end:
        return [(start, 0xFFFF)]
    window = (end - start) + 1
    bit_length = int(math.floor(math.log2(window)))

    def get_range(e, bl):
        rl = (1 << bl) - 1
        rs = e & ~rl & 0xFFFF
        return rs, rs + rl

    rs, re_ = get_range(end, bit_length)
    while re_ > end:
        bit_length -= 1
        rs, re_ = get_range(end, bit_length)
    current = (rs, 0xFFFF ^ ((1 << bit_length) - 1))
    out = []
    if start != rs:
        out += bitwise_match(start, rs - 1)
    out.append(current)
    if end != re_:
        out += bitwise_match(re_ + 1, end)
    return out


def ports_to_bit_ranges(port: Optional[int], end_port: Optional[int]):
    """network_policy.go:986-1017. BitRange = (value, mask|None)."""
    if end_port is not None and port is not None and end_port > port:
        return [(v, m) for v, m in bitwise_match(port, end_port)]
    if port is not None:
        return [(port, None)]
    return [(0, None)]


def get_service_match_pairs(svc: dict, ip_protocols: List[str]):
    """network_policy.go:891-983."""
    out = []
    dst_ranges = ports_to_bit_ranges(svc.get("port"), svc.get("end_port"))
    src_ranges = None
    if svc.get("src_port") is not None:
        src_ranges = ports_to_bit_ranges(svc.get("src_port"), svc.get("src_end_port"))

    def add_l4(dkey, skey):
        for br in dst_ranges:
            pairs = [(dkey, ("bitrange", br[0], br[1]))]
            if src_ranges is not None:
                # Go appends to the same backing slice for each src range (network_policy.go:902-906);
                # every appended flow therefore carries the dst pair plus ALL src pairs up to that point.
                # With a single src range (the only form the API produces) this is just [dst, src].
                for sr in src_ranges:
                    pairs = pairs + [(skey, ("bitrange", sr[0], sr[1]))]
                    out.append(list(pairs))
            else:
                out.append(pairs)

    proto = svc.get("protocol")
    if proto == "TCP":
        for ipp in ip_protocols:
            add_l4(MatchTCPDstPort, MatchTCPSrcPort) if ipp == "ip" else add_l4(MatchTCPv6DstPort, MatchTCPv6SrcPort)
    elif proto == "UDP":
        for ipp in ip_protocols:
            add_l4(MatchUDPDstPort, MatchUDPSrcPort) if ipp == "ip" else add_l4(MatchUDPv6DstPort, MatchUDPv6SrcPort)
    elif proto == "SCTP":
        for ipp in ip_protocols:
            add_l4(MatchSCTPDstPort, MatchSCTPSrcPort) if ipp == "ip" else add_l4(MatchSCTPv6DstPort, MatchSCTPv6SrcPort)
    elif proto == "ICMP":
        for ipp in ip_protocols:
            tkey, ckey = (MatchICMPType, MatchICMPCode) if ipp == "ip" else (MatchICMPv6Type, MatchICMPv6Code)
            pairs = []
            if svc.get("icmp_type") is not None:
                pairs.append((tkey, ("icmp", svc["icmp_type"])))
            if svc.get("icmp_code") is not None:
                pairs.append((ckey, ("icmp", svc["icmp_code"])))
            if not pairs:
                pairs.append((tkey, ("icmp", None)))
            out.append(pairs)
    elif proto == "IGMP":
        if svc.get("igmp_type") == 0x11:  # crdv1beta1.IGMPQuery
            ga = svc.get("group_address") or "224.0.0.1"  # types.McastAllHosts
            out.append([(MatchDstIP, ("ip", ipaddress.ip_address(ga))), (MatchIGMPProtocol, ("int", 0))])
    else:
        add_l4(MatchTCPDstPort, MatchTCPSrcPort)
    return out


# ---------------------------------------------------------------------------------------------
# flows
# ---------------------------------------------------------------------------------------------
@dataclass
class Flow:
    table: str
    priority: int
    match: Dict[str, tuple] = field(default_factory=dict)
    actions: List[tuple] = field(default_factory=list)
    cookie: int = 0

    def copy_with_priority(self, p):
        return Flow(self.table, p, dict(self.match), list(self.actions), self.cookie)


def _set_proto(m, proto):
    """ofFlowBuilder.MatchProtocol (pkg/ovs/openflow/ofctrl_builder.go:408-446): ethertype is
    overwritten, the IP protocol is only set by protocols that carry one."""
    m["dl_type"] = PROTO_ETH[proto]
    if proto in PROTO_NUM:
        m["nw_proto"] = PROTO_NUM[proto]


def _ct_new(m, new: bool):
    data, mask = m.get("ct_state", (0, 0))
    mask |= 1
    data = (data | 1) if new else (data & ~1)
    m["ct_state"] = (data, mask)


def add_flow_match(m: dict, key: MatchKey, value):
    """featureNetworkPolicy.addFlowMatch (pipeline.go:1896-2000)."""
    tag = value[0]
    if key is MatchDstOFPort:
        m["reg1"] = (value[1], None)
    elif key is MatchSrcOFPort:
        m["in_port"] = (value[1], None)
    elif key in (MatchDstIP, MatchDstIPv6, MatchSrcIP, MatchSrcIPv6,
                 MatchDstIPNet, MatchDstIPNetv6, MatchSrcIPNet, MatchSrcIPNetv6):
        _set_proto(m, key.proto)
        fld = key.key
        if tag == "ip":
            m[fld] = (int(value[1]), None, value[1].version)
        else:
            n = value[1]
            m[fld] = (int(n.network_address), n.prefixlen, n.version)
    elif key in (MatchCTDstIP, MatchCTDstIPv6, MatchCTSrcIP, MatchCTSrcIPv6,
                 MatchCTDstIPNet, MatchCTDstIPNetv6, MatchCTSrcIPNet, MatchCTSrcIPNetv6):
        _ct_new(m, True)
        _set_proto(m, key.proto)
        if tag == "ip":
            m[key.key] = (int(value[1]), None, value[1].version)
        else:
            n = value[1]
            m[key.key] = (int(n.network_address), n.prefixlen, n.version)
    elif key.category == "L4PortAddr":
        _set_proto(m, key.proto)
        v, mask = value[1], value[2]
        if v > 0:
            m[key.key] = (v, mask)
    elif key.category == "ICMPAddr":
        _set_proto(m, key.proto)
        if value[1] is not None:
            m[key.key.replace("icmpv6", "icmp")] = (value[1], None)
    elif key is MatchServiceGroupID:
        m["reg7"] = (value[1], None)
    elif key is MatchIGMPProtocol:
        _set_proto(m, key.proto)
    elif key is MatchLabelID:
        m["tun_id"] = (value[1], None)
    elif key is MatchCTState:
        d, mk = value[1], value[2]
        od, om = m.get("ct_state", (0, 0))
        m["ct_state"] = ((od & ~mk) | d, om | mk)
    else:
        raise ValueError("unsupported match key %s" % key.name)


# ---------------------------------------------------------------------------------------------
# text format (pkg/ovs/openflow/utils.go)
# ---------------------------------------------------------------------------------------------
_CT_STATES = ["new", "est", "rel", "rpl", "inv", "trk", "snat", "dnat"]


def _proto_str(eth, nwp):
    # utils.go:298-354 matchProtoToString
    table = {(0x0800, 0): "ip", (0x86DD, 0): "ipv6", (0x0806, 0): "arp",
             (0x0800, 6): "tcp", (0x86DD, 6): "tcp6", (0x0800, 17): "udp", (0x86DD, 17): "udp6",
             (0x0800, 132): "sctp", (0x86DD, 132): "sctp6", (0x0800, 1): "icmp", (0x86DD, 58): "icmp6",
             (0x0800, 2): "igmp"}
    return table.get((eth, nwp or 0), "")


def _ip_str(v):
    value, plen, ver = v
    ip = ipaddress.ip_address(value) if ver == 4 else ipaddress.IPv6Address(value)
    full = 32 if ver == 4 else 128
    if plen is not None and plen < full:
        return "%s/%d" % (ip, plen)
    return str(ip)


def _hex_label(v):
    return "0x%x" % v


def match_to_string(f: Flow) -> str:
    """getFlowModMatch (utils.go:905-1098): fixed field order."""
    m = f.match
    parts = ["priority=%d" % f.priority]
    if "conj_id" in m:
        parts.append("conj_id=%d" % m["conj_id"][0])
    if "ct_state" in m:
        d, mk = m["ct_state"]
        s = ""
        for i in range(8):
            if mk & (1 << i):
                s += ("+" if d & (1 << i) else "-") + _CT_STATES[i]
        parts.append("ct_state=" + s)
    if "ct_mark" in m:
        d, mk = m["ct_mark"]
        parts.append("ct_mark=0x%x/0x%x" % (d, mk) if mk is not None and mk != 0xFFFFFFFF else "ct_mark=0x%x" % d)
    if "ct_label" in m:
        d, mk = m["ct_label"]
        parts.append("ct_label=0x%x/0x%x" % (d, mk) if mk != (1 << 128) - 1 else "ct_label=0x%x" % d)
    for fld in ("ct_nw_src", "ct_nw_dst", "ct_ipv6_src", "ct_ipv6_dst"):
        if fld in m:
            parts.append("%s=%s" % (fld, _ip_str(m[fld])))
    if "dl_type" in m:
        parts.append(_proto_str(m["dl_type"], m.get("nw_proto")))
    for i in range(16):
        r = "reg%d" % i
        if r in m:
            v, mk = m[r]
            if mk is None or mk == 0xFFFFFFFF:
                parts.append("%s=0x%x" % (r, v))
            else:
                parts.append("%s=0x%x/0x%x" % (r, v, mk))
    if "tun_id" in m:
        parts.append("tun_id=%d" % m["tun_id"][0])
    if "in_port" in m:
        parts.append("in_port=%d" % m["in_port"][0])
    for fld in ("nw_src", "nw_dst", "ipv6_src", "ipv6_dst"):
        if fld in m:
            parts.append("%s=%s" % (fld, _ip_str(m[fld])))
    if "icmp_type" in m:
        parts.append("icmp_type=%d" % m["icmp_type"][0])
    if "icmp_code" in m:
        parts.append("icmp_code=%d" % m["icmp_code"][0])
    for fld in ("tp_src", "tp_dst"):
        if fld in m:
            v, mk = m[fld]
            if mk is None or mk == 0xFFFF:
                parts.append("%s=%d" % (fld, v))
            else:
                parts.append("%s=0x%x/0x%x" % (fld, v, mk))
    return ",".join(parts)


def _action_to_string(a) -> str:
    kind = a[0]
    if kind == "conjunction":
        return "conjunction(%d,%d/%d)" % (a[1], a[2], a[3])
    if kind == "set_reg":          # ("set_reg", reg, value, mask|None)
        _, reg, v, mk = a
        if mk is None:
            return "set_field:0x%x->reg%d" % (v, reg)
        return "set_field:0x%x/0x%x->reg%d" % (v, mk, reg)
    if kind == "ct_commit":        # ("ct_commit", table, zone, [(label_v, label_m)])
        _, table, zone, labels = a
        execs = ",".join("set_field:%s/0x%x->ct_label" % (_hex_label(v), mk) for v, mk in labels)
        s = "ct(commit,table=%s,zone=%d" % (table, zone)
        if execs:
            s += ",exec(%s)" % execs
        return s + ")"
    if kind == "goto_table":
        return "goto_table:%s" % a[1]
    if kind == "group":
        return "group:%d" % a[1]
    if kind == "drop":
        return "drop"
    if kind == "meter":            # ("meter", id)                       utils.go:623
        return "meter:%d" % a[1]
    if kind == "controller":       # ("controller", userdata bytes)      utils.go:800-838
        return "controller(id=%d,reason=no_match,userdata=%s,max_len=65535)" % (
            CONTROLLER_ID, ".".join("%02x" % b for b in a[1]))
    raise ValueError(kind)


def flow_to_string(f: Flow) -> str:
    """FlowModToString (utils.go:1222-1224)."""
    base = ("cookie=0x%x, " % f.cookie if f.cookie else "") + "table=%s" % f.table
    acts = [_action_to_string(a) for a in f.actions if a[0] != "drop"]
    astr = "actions=" + (",".join(acts) if acts else "drop")
    return "%s, %s %s" % (base, match_to_string(f), astr)


def flow_dump_key(f: Flow) -> str:
    """getFlowDumpKey (pipeline.go:385-387, utils.go:1226-1242): the match without its priority,
    prefixed by the table (named here: the build has no numeric OVS table ids)."""
    parts = [p for p in match_to_string(f).split(",") if not p.startswith("priority")]
    return "table=%s,%s" % (f.table, ",".join(parts))


def flow_identity(f: Flow):
    """(table, priority, match) -- what OVS keys a flow by."""
    return (f.table, f.priority, match_to_string(f).split(",", 1)[1] if "," in match_to_string(f) else "")


# ---------------------------------------------------------------------------------------------
# conjunctive match state (network_policy.go:325-695)
# ---------------------------------------------------------------------------------------------
@dataclass
class ConjunctiveMatch:
    table: str
    priority: Optional[int]
    pairs: List[tuple]

    def key(self) -> str:
        p = PRIORITY_NORMAL if self.priority is None else self.priority
        return "table:%s,priority:%d,matchPair:%s" % (
            self.table, p, ",".join(match_pair_key_string(k, v) for k, v in self.pairs))


@dataclass
class ConjAction:
    conj_id: int
    clause_id: int
    n_clause: int


class Context:
    """conjMatchFlowContext (network_policy.go:442-461)."""

    def __init__(self, match: ConjunctiveMatch, feature, enable_logging):
        self.match = match
        self.actions: Dict[int, ConjAction] = {}
        self.deny_all: Dict[int, bool] = {}
        self.feature = feature
        self.flow: Optional[Flow] = None
        self.drop_flow: Optional[Flow] = None
        self.drop_flow_enable_logging = enable_logging


class Clause:
    def __init__(self, action: ConjAction, rule_table: str, drop_table: Optional[str]):
        self.action = action
        self.matches: Dict[str, Context] = {}
        self.rule_table = rule_table
        self.drop_table = drop_table


class Conjunction:
    """policyRuleConjunction (network_policy.go:664-677)."""

    def __init__(self, cid):
        self.id = cid
        self.from_clause: Optional[Clause] = None
        self.to_clause: Optional[Clause] = None
        self.service_clause: Optional[Clause] = None
        self.action_flows: List[Flow] = []
        self.metric_flows: List[Flow] = []
        self.np_ref = None
        self.rule_name = ""
        self.rule_table = ""
        self.rule_log_label = ""
        self.tier_priority = None
        self.action = None

    def clauses(self):
        return [c for c in (self.from_clause, self.to_clause, self.service_clause) if c is not None]

    def action_flow_priorities(self):
        return [str(f.priority) for f in self.action_flows]


class _PolicyCache(dict):
    """policyCache (network_policy.go:2080) plus an index (rule table, action-flow priority) -> conj
    ids, so UninstallPolicyRuleFlows' stale-priority check and ReassignFlowPriorities look rules up
    by priority instead of scanning all of them (C5 replays hundreds of both over 100k rules)."""

    def __init__(self):
        super().__init__()
        self.by_prio: Dict[tuple, set] = {}

    def index(self, conj, add: bool):
        for f in conj.action_flows:
            k = (conj.rule_table, f.priority)
            if add:
                self.by_prio.setdefault(k, set()).add(conj.id)
            elif k in self.by_prio:
                self.by_prio[k].discard(conj.id)

    def __setitem__(self, key, conj):
        old = self.get(key)
        if old is not None:
            self.index(old, False)
        super().__setitem__(key, conj)
        self.index(conj, True)

    def __delitem__(self, key):
        self.index(self[key], False)
        super().__delitem__(key)

    def with_priority(self, table: str, priority: int) -> list:
        return [self[c] for c in sorted(self.by_prio.get((table, priority), ())) if c in self]


class ConjunctionNotFound(Exception):
    """network_policy.go:309-319."""

    def __init__(self, cid):
        super().__init__("policyRuleConjunction with ID %d not found" % cid)
        self.conj_id = cid


def _contains_label_identity(addrs) -> bool:
    """containsLabelIdentityAddress (network_policy.go:1491-1500)."""
    return any((a if isinstance(a, tuple) else parse_address(a))[0] == "labelid" for a in (addrs or []))


class FeatureNetworkPolicy:
    """featureNetworkPolicy (network_policy.go:2067-2142) with the flow table it would have
    realized on OVS (the `installed` map stands in for ovs-vswitchd's flow table)."""

    def __init__(self, ipv4=True, ipv6=False, enable_antrea_policy=True, enable_deny_tracking=False,
                 cookie=0x1020000000000, bundle_fail=False, ovs_meters=False, k8s_node=True):
        self.ip_protocols = (["ip"] if ipv4 else []) + (["ipv6"] if ipv6 else [])
        self.ovs_meters = ovs_meters
        self.k8s_node = k8s_node
        self.enable_antrea_policy = enable_antrea_policy
        self.enable_deny_tracking = enable_deny_tracking
        self.cookie = cookie
        self.global_cache: Dict[str, Context] = {}
        self.policy_cache: Dict[int, Conjunction] = _PolicyCache()
        self.egress_tables = {"EgressRule", "EgressDefaultRule"}
        if enable_antrea_policy:
            self.egress_tables.add("AntreaPolicyEgressRule")
        # ovs flow table stand-in: identity -> Flow
        self.installed: Dict[tuple, Flow] = {}
        self.bundle_fail = bundle_fail
        self.bundles = 0

    # ----- OVS stand-in -----------------------------------------------------------------
    def _apply(self, add=(), mod=(), delete=()):
        """Bridge.AddFlowsInBundle: all-or-nothing (ofctrl_bridge.go:468-539)."""
        if self.bundle_fail:
            raise RuntimeError("bundle failed")
        self.bundles += 1
        for f in delete:
            self.installed.pop(flow_identity(f), None)
        for f in list(add) + list(mod):
            self.installed[flow_identity(f)] = f

    def init_flows(self) -> List[Flow]:
        """featureNetworkPolicy.initFlows (network_policy.go:2126-2142): ingressClassifierFlows on a K8s
        Node (pipeline.go:2144-2182), skipPolicyRuleCheckFlows (:2167-2211), initLoggingFlows
        (:2249-2269)."""
        flows = []
        if self.k8s_node:
            for mark in (TO_GATEWAY, TO_TUNNEL, TO_UPLINK):
                flows.append(Flow("IngressSecurityClassifier", PRIORITY_NORMAL, {"reg0": (mark, 0xF0)},
                                  [("goto_table", "IngressMetric")], self.cookie))
            flows.append(Flow("IngressSecurityClassifier", PRIORITY_NORMAL, {"ct_mark": (HAIRPIN_CT_MARK, HAIRPIN_CT_MARK)},
                              [("goto_table", "ConntrackCommit")], self.cookie))
        flows += self.skip_flows()
        for ops in range(1, 8):  # logging + store-deny + reject operations
            acts = [("meter", PACKET_IN_METER_NP)] if self.ovs_meters else []
            acts.append(("controller", (PACKET_IN_CATEGORY_NP, ops)))
            flows.append(Flow("Output", PRIORITY_NORMAL, {"reg0": ((ops << 25) | (2 << 21), 0xFE600000)}, acts,
                              self.cookie))
        return flows

    def skip_flows(self) -> List[Flow]:
        """skipPolicyRuleCheckFlows (network_policy.go:2167-2211)."""
        flows = []
        eg, ing, prio = "EgressRule", "IngressRule", PRIORITY_HIGH
        if self.enable_antrea_policy:
            eg, ing, prio = "AntreaPolicyEgressRule", "AntreaPolicyIngressRule", PRIORITY_TOP_ANTREA_POLICY
        for ipp in self.ip_protocols:
            for tbl, metric in ((eg, "EgressMetric"), (ing, "IngressMetric")):
                for bit in (1, 2):  # est, rel
                    m = {}
                    _set_proto(m, ipp)
                    m["ct_state"] = (1 << bit, 1 | (1 << bit))
                    flows.append(Flow(tbl, prio, m, [("goto_table", metric)], self.cookie))
        return flows

    def initialize(self):
        self._apply(add=self.init_flows())

    def dump_flows(self) -> List[str]:
        return [flow_to_string(f) for f in self.installed.values()]

    # ----- flow builders (pipeline.go) ----------------------------------------------------
    def conjunctive_match_flow(self, table, pairs, priority, actions: List[ConjAction]) -> Flow:
        """pipeline.go:2019-2037; conjunction actions ordered by id (deterministic mode)."""
        m = {}
        for k, v in pairs:
            add_flow_match(m, k, v)
        acts = [("conjunction", a.conj_id, a.clause_id, a.n_clause)
                for a in sorted(actions, key=lambda a: (a.conj_id, a.clause_id))]
        return Flow(table, PRIORITY_NORMAL if priority is None else priority, m, acts, self.cookie)

    def default_drop_flow(self, table, pairs, enable_logging) -> Flow:
        """pipeline.go:2040-2065."""
        m = {}
        for k, v in pairs:
            add_flow_match(m, k, v)
        if enable_logging or self.enable_deny_tracking:
            ops = (1 if enable_logging else 0) + (2 if self.enable_deny_tracking else 0)
            acts = [("set_reg", 0, DISPOSITION_DROP << 11, 0x1800), ("set_reg", 0, ops << 25, 0x1FE000000 & 0xFFFFFFFF),
                    ("set_reg", 0, 2 << 21, 0x600000), ("set_reg", 2, TABLE_NUM[table], 0xFF), ("goto_table", "Output")]
            return Flow(table, PRIORITY_NORMAL, m, acts, self.cookie)
        return Flow(table, PRIORITY_NORMAL, m, [("drop",)], self.cookie)

    def mcnp_drop_flow(self, table, pairs) -> Flow:
        """pipeline.go:2068-2076."""
        m = {}
        add_flow_match(m, MatchLabelID, ("int", UNKNOWN_LABEL_IDENTITY))
        for k, v in pairs:
            add_flow_match(m, k, v)
        return Flow(table, PRIORITY_NORMAL, m, [("drop",)], self.cookie)

    def conjunction_action_flows(self, cid, table, next_table, priority, enable_logging) -> List[Flow]:
        """pipeline.go:1718-1808 (unicast; L7 redirect not modeled)."""
        p = PRIORITY_LOW if priority is None else priority
        egress = table in self.egress_tables
        reg = 5 if egress else 6
        label = (cid << 32, 0xFFFFFFFF00000000) if egress else (cid, 0xFFFFFFFF)
        flows = []
        for ipp in self.ip_protocols:
            m = {"conj_id": (cid,)}
            _set_proto(m, ipp)
            zone = CT_ZONE_V6 if ipp == "ipv6" else CT_ZONE
            acts = [("set_reg", reg, cid, None), ("ct_commit", next_table, zone, [label])]
            if enable_logging:
                acts += [("set_reg", 0, 0, 0x1800), ("set_reg", 0, 2 << 21, 0x600000),
                         ("set_reg", 0, 1 << 25, 0x1FE000000 & 0xFFFFFFFF), ("set_reg", 2, TABLE_NUM[table], 0xFF),
                         ("goto_table", "Output")]
            flows.append(Flow(table, p, m, acts, self.cookie))
        return flows

    def conjunction_deny_flow(self, cid, table, priority, disposition, enable_logging) -> Flow:
        """pipeline.go:1812-1859."""
        metric = "EgressMetric" if table in self.egress_tables else "IngressMetric"
        m = {"conj_id": (cid,)}
        acts = [("set_reg", 3, cid, None), ("set_reg", 0, 0x400, 0x400)]
        ops = 0
        if self.enable_deny_tracking:
            ops += 2
            acts.append(("set_reg", 0, disposition << 11, 0x1800))
        if enable_logging:
            ops += 1
            acts.append(("set_reg", 0, disposition << 11, 0x1800))
        if disposition == DISPOSITION_REJ:
            ops += 4
        if enable_logging or self.enable_deny_tracking or disposition == DISPOSITION_REJ:
            acts += [("set_reg", 0, ops << 25, 0x1FE000000 & 0xFFFFFFFF), ("set_reg", 2, TABLE_NUM[table], 0xFF),
                     ("group", LOGGING_GROUP[metric])]
        else:
            acts.append(("goto_table", metric))
        return Flow(table, priority, m, acts, self.cookie)

    def conjunction_pass_flow(self, cid, table, priority, enable_logging) -> Flow:
        """pipeline.go:1861-1886."""
        egress = table in self.egress_tables
        reg = 5 if egress else 6
        nxt = "EgressRule" if egress else "IngressRule"
        m = {"conj_id": (cid,)}
        acts = [("set_reg", reg, cid, None)]
        if enable_logging:
            acts += [("set_reg", 0, DISPOSITION_PASS << 11, 0x1800), ("set_reg", 0, 1 << 25, 0xFE000000),
                     ("set_reg", 2, TABLE_NUM[table], 0xFF), ("group", LOGGING_GROUP[nxt])]
        else:
            acts.append(("goto_table", nxt))
        return Flow(table, priority, m, acts, self.cookie)

    def allow_metric_flows(self, cid, ingress) -> List[Flow]:
        """pipeline.go:1604-1651."""
        metric = "IngressMetric" if ingress else "EgressMetric"
        label = (cid, 0xFFFFFFFF) if ingress else (cid << 32, 0xFFFFFFFF00000000)
        flows = []
        for ipp in self.ip_protocols:
            for new in (True, False):
                m = {}
                _set_proto(m, ipp)
                _ct_new(m, new)
                m["ct_label"] = label
                flows.append(Flow(metric, PRIORITY_NORMAL, m, [("goto_table", NEXT_TABLE[metric])], self.cookie))
        return flows

    def deny_metric_flow(self, cid, ingress) -> Flow:
        """pipeline.go:1653-1670."""
        metric = "IngressMetric" if ingress else "EgressMetric"
        m = {"reg0": (0x400, 0x400), "reg3": (cid, None)}
        return Flow(metric, PRIORITY_NORMAL, m, [("drop",)], self.cookie)

    # ----- clause logic (network_policy.go:791-1126, 1408-1489) ---------------------------
    def _add_conjunctive_match_flow(self, clause: Clause, match: ConjunctiveMatch, enable_logging, is_mcnp):
        """clause.addConjunctiveMatchFlow (network_policy.go:791-864). Returns a change record."""
        key = match.key()
        if key in clause.matches:
            return None
        ctx = self.global_cache.get(key)
        ctx_type = "modification"
        drop_change = None
        if ctx is None:
            ctx = Context(match, self, enable_logging)
            ctx_type = "insertion"
            if clause.drop_table is not None and ctx.drop_flow is None:
                if is_mcnp:
                    drop_change = ("insertion", self.mcnp_drop_flow(clause.drop_table, match.pairs))
                else:
                    drop_change = ("insertion", self.default_drop_flow(clause.drop_table, match.pairs, enable_logging))
        elif ctx.drop_flow_enable_logging != enable_logging:
            ctx.drop_flow_enable_logging = enable_logging
            if clause.drop_table is not None and ctx.drop_flow is not None:
                drop_change = ("modification", self.default_drop_flow(clause.drop_table, match.pairs, enable_logging))
        ch = {"ctx": ctx, "ctx_type": ctx_type, "clause": clause, "act_type": "insertion", "act": None,
              "match_flow": None, "drop": drop_change, "key": key}
        if clause.action.n_clause > 1:
            if clause.action.conj_id not in ctx.actions:
                acts = [clause.action] + list(ctx.actions.values())
                flow = self.conjunctive_match_flow(match.table, match.pairs, match.priority, acts)
                ch["match_flow"] = ("insertion" if ctx.flow is None else "modification", flow)
                ch["act"] = clause.action
        else:
            ch["match_flow"] = ("insertion", None)
        return ch

    def _delete_conjunctive_match_flow(self, clause: Clause, key: str):
        """clause.deleteConjunctiveMatchFlow (network_policy.go:1049-1098)."""
        ctx = clause.matches.get(key)
        if ctx is None:
            return None
        ch = {"ctx": ctx, "ctx_type": "modification", "clause": clause, "act_type": "deletion", "act": None,
              "match_flow": None, "drop": None, "key": key}
        cid = clause.action.conj_id
        n_actions = len(ctx.actions)
        n_deny = len(ctx.deny_all)
        if clause.action.n_clause > 1:
            if cid in ctx.actions:
                if n_actions == 1 and ctx.flow is not None:
                    ch["match_flow"] = ("deletion", ctx.flow)
                else:
                    acts = [a for a in ctx.actions.values() if a.conj_id != cid]
                    flow = self.conjunctive_match_flow(ctx.match.table, ctx.match.pairs, ctx.match.priority, acts)
                    ch["match_flow"] = ("insertion" if ctx.flow is None else "modification", flow) if acts else None
                ch["act"] = ctx.actions[cid]
                n_actions -= 1
        else:
            ch["match_flow"] = ("deletion", None)
            n_deny -= 1
        if n_actions == 0 and n_deny == 0:
            if ctx.drop_flow is not None:
                ch["drop"] = ("deletion", ctx.drop_flow)
            ch["ctx_type"] = "deletion"
        return ch

    def _update_context_status(self, ch):
        """conjMatchFlowContextChange.updateContextStatus (network_policy.go:583-646)."""
        ctx, clause = ch["ctx"], ch["clause"]
        key = ctx.match.key()
        act = ch["act"]
        if ch["act_type"] == "insertion":
            clause.matches[key] = ctx
            if act is not None:
                ctx.actions[act.conj_id] = act
        else:
            clause.matches.pop(key, None)
            if act is not None:
                ctx.actions.pop(act.conj_id, None)
        mf = ch["match_flow"]
        if mf is not None:
            typ, flow = mf
            if typ in ("insertion", "modification"):
                if flow is not None:
                    ctx.flow = flow
                else:
                    if ch["act_type"] == "insertion":
                        ctx.deny_all[clause.action.conj_id] = True
                    else:
                        ctx.deny_all.pop(clause.action.conj_id, None)
            else:
                if flow is not None:
                    ctx.flow = None
                else:
                    ctx.deny_all.pop(clause.action.conj_id, None)
        if ch["drop"] is not None:
            typ, flow = ch["drop"]
            if typ == "insertion":
                ctx.drop_flow = flow
            elif typ == "deletion":
                ctx.drop_flow = None
        if ch["ctx_type"] == "insertion":
            self.global_cache[key] = ctx
        elif ch["ctx_type"] == "deletion":
            self.global_cache.pop(key, None)

    def _apply_changes(self, changes):
        """applyConjunctiveMatchFlows + sendConjunctiveFlows (network_policy.go:1359-1396)."""
        add, mod, dele = [], [], []
        for ch in changes:
            for fc in (ch["match_flow"], ch["drop"]):
                if fc is None or fc[1] is None:
                    continue
                {"insertion": add, "modification": mod, "deletion": dele}[fc[0]].append(fc[1])
        self._apply(add, mod, dele)
        for ch in changes:
            self._update_context_status(ch)

    def calculate_clauses(self, conj: Conjunction, rule: dict):
        """policyRuleConjunction.calculateClauses (network_policy.go:1423-1472)."""
        egress = rule["direction"] == "Out"
        drop_table = "EgressDefaultRule" if egress else "IngressDefaultRule"
        rule_table = rule["table"]
        is_anp = rule.get("policy_type", K8S_NP) != K8S_NP
        frm, to, svc = rule.get("from"), rule.get("to"), rule.get("service")
        n = 0
        fid = tid = sid = 0
        if frm is not None:
            n += 1
            fid = n
        if to is not None:
            n += 1
            tid = n
        if svc is not None:
            n += 1
            sid = n
        if frm is not None:
            dt = None if (not egress or is_anp) else drop_table
            conj.from_clause = Clause(ConjAction(conj.id, fid, n), rule_table, dt)
        if to is not None:
            dt = None if (egress or (is_anp and not _contains_label_identity(frm))) else drop_table
            conj.to_clause = Clause(ConjAction(conj.id, tid, n), rule_table, dt)
        if svc is not None:
            conj.service_clause = Clause(ConjAction(conj.id, sid, n), rule_table, None)
        return n, rule_table, drop_table

    def calculate_action_flows(self, rule: dict) -> Optional[Conjunction]:
        """calculateActionFlowChangesForRule (network_policy.go:1186-1228)."""
        cid = rule["flow_id"]
        if cid in self.policy_cache:
            return None
        conj = Conjunction(cid)
        conj.np_ref = (rule.get("policy_type", K8S_NP), rule.get("policy_namespace", ""),
                       rule.get("policy_name", ""), rule.get("policy_uid", ""))
        conj.rule_name = rule.get("name", "")
        conj.rule_log_label = rule.get("log_label", "")
        conj.tier_priority = rule.get("tier_priority")
        n, rule_table, drop_table = self.calculate_clauses(conj, rule)
        conj.rule_table = rule_table
        ingress = rule_table not in self.egress_tables
        is_anp = rule.get("policy_type", K8S_NP) != K8S_NP
        action = rule.get("action")
        conj.action = action if is_anp else "Allow"
        logging = bool(rule.get("enable_logging"))
        prio = rule.get("priority")
        if n > 1:
            if is_anp and action == "Drop":
                conj.metric_flows = [self.deny_metric_flow(cid, ingress)]
                conj.action_flows = [self.conjunction_deny_flow(cid, rule_table, prio, DISPOSITION_DROP, logging)]
            elif is_anp and action == "Reject":
                conj.metric_flows = [self.deny_metric_flow(cid, ingress)]
                conj.action_flows = [self.conjunction_deny_flow(cid, rule_table, prio, DISPOSITION_REJ, logging)]
            elif is_anp and action == "Pass":
                conj.action_flows = [self.conjunction_pass_flow(cid, rule_table, prio, logging)]
            else:
                conj.metric_flows = self.allow_metric_flows(cid, ingress)
                conj.action_flows = self.conjunction_action_flows(cid, rule_table, NEXT_TABLE[drop_table], prio, logging)
        return conj

    def _rule_matches(self, conj: Conjunction, rule: dict):
        """The (clause, match) pairs of a rule, in the order calculateChangesForRuleCreation visits them."""
        out = []
        prio = rule.get("priority")
        if conj.from_clause is not None:
            for a in rule["from"]:
                a = parse_address(a)
                out.append((conj.from_clause, ConjunctiveMatch(conj.from_clause.rule_table, prio,
                                                               [(address_match_key(a, True), address_match_value(a))])))
        if conj.to_clause is not None:
            for a in rule["to"]:
                a = parse_address(a)
                out.append((conj.to_clause, ConjunctiveMatch(conj.to_clause.rule_table, prio,
                                                             [(address_match_key(a, False), address_match_value(a))])))
        if conj.service_clause is not None:
            for svc in rule["service"]:
                for pairs in get_service_match_pairs(svc, self.ip_protocols):
                    out.append((conj.service_clause, ConjunctiveMatch(conj.service_clause.rule_table, prio, pairs)))
        return out

    # ----- openflow.Client NP surface ----------------------------------------------------
    def install_policy_rule_flows(self, rule: dict):
        """InstallPolicyRuleFlows (network_policy.go:1160-1183)."""
        conj = self.calculate_action_flows(rule)
        if conj is None:
            return
        is_mcnp = _contains_label_identity([parse_address(a) for a in (rule.get("from") or [])])
        changes = []
        for clause, match in self._rule_matches(conj, rule):
            ch = self._add_conjunctive_match_flow(clause, match, bool(rule.get("enable_logging")), is_mcnp)
            if ch is not None:
                changes.append(ch)
        self._apply(add=conj.metric_flows + conj.action_flows)
        self._apply_changes(changes)
        self.policy_cache[conj.id] = conj

    def batch_install_policy_rule_flows(self, rules: List[dict]):
        """BatchInstallPolicyRuleFlows (network_policy.go:1310-1356)."""
        all_flows, conjs = [], []
        for rule in rules:
            conj = self.calculate_action_flows(rule)
            if conj is None:
                continue
            is_mcnp = _contains_label_identity([parse_address(a) for a in (rule.get("from") or [])])
            for clause, match in self._rule_matches(conj, rule):
                key = match.key()
                if key in clause.matches:
                    continue
                ctx = self.global_cache.get(key)
                if ctx is None:
                    ctx = Context(match, self, bool(rule.get("enable_logging")))
                    if clause.drop_table is not None:
                        ctx.drop_flow = (self.mcnp_drop_flow(clause.drop_table, match.pairs) if is_mcnp else
                                         self.default_drop_flow(clause.drop_table, match.pairs,
                                                                bool(rule.get("enable_logging"))))
                    self.global_cache[key] = ctx
                clause.matches[key] = ctx
                if clause.action.n_clause > 1:
                    ctx.actions[clause.action.conj_id] = clause.action
                else:
                    ctx.deny_all[clause.action.conj_id] = True
            all_flows += conj.action_flows + conj.metric_flows
            conjs.append(conj)
        for ctx in self.global_cache.values():
            if ctx.actions:
                ctx.flow = self.conjunctive_match_flow(ctx.match.table, ctx.match.pairs, ctx.match.priority,
                                                       list(ctx.actions.values()))
                all_flows.append(ctx.flow)
            if ctx.drop_flow is not None:
                all_flows.append(ctx.drop_flow)
        try:
            self._apply(add=all_flows)
        except RuntimeError:
            self.global_cache = {}
            raise
        for conj in conjs:
            self.policy_cache[conj.id] = conj
        return all_flows

    def uninstall_policy_rule_flows(self, rule_id: int) -> List[str]:
        """UninstallPolicyRuleFlows (network_policy.go:1570-1624)."""
        conj = self.policy_cache.get(rule_id)
        if conj is None:
            return []
        stale = self._stale_priorities(conj)
        self._apply(delete=conj.action_flows + conj.metric_flows)
        changes = []
        for cl in conj.clauses():
            for key in list(cl.matches.keys()):
                ch = self._delete_conjunctive_match_flow(cl, key)
                if ch is not None:
                    changes.append(ch)
        self._apply_changes(changes)
        del self.policy_cache[rule_id]
        return stale

    def _stale_priorities(self, conj):
        if conj.rule_table in ("IngressRule", "EgressRule"):
            return []
        stale = []
        for f in conj.action_flows:
            p = str(f.priority)
            if not any(c.id != conj.id for c in self.policy_cache.with_priority(conj.rule_table, f.priority)):
                stale.append(p)
        return stale

    def _address_clause(self, conj, addr_type):
        return conj.from_clause if addr_type == "src" else conj.to_clause

    def add_policy_rule_address(self, rule_id, addr_type, addresses, priority=None, enable_logging=False,
                                is_mcnp=False):
        """AddPolicyRuleAddress (network_policy.go:1661-1682)."""
        conj = self.policy_cache.get(rule_id)
        if conj is None:
            raise ConjunctionNotFound(rule_id)
        clause = self._address_clause(conj, addr_type)
        if clause is None:
            raise ValueError("no clause is using addrType %d" % (0 if addr_type == "src" else 1))
        changes = []
        for a in addresses:
            a = parse_address(a)
            m = ConjunctiveMatch(clause.rule_table, priority,
                                 [(address_match_key(a, addr_type == "src"), address_match_value(a))])
            ch = self._add_conjunctive_match_flow(clause, m, enable_logging, is_mcnp)
            if ch is not None:
                changes.append(ch)
        self._apply_changes(changes)

    def delete_policy_rule_address(self, rule_id, addr_type, addresses, priority=None):
        """DeletePolicyRuleAddress (network_policy.go:1686-1710)."""
        conj = self.policy_cache.get(rule_id)
        if conj is None:
            raise ConjunctionNotFound(rule_id)
        clause = self._address_clause(conj, addr_type)
        if clause is None:
            raise ValueError("no clause is using addrType %d" % (0 if addr_type == "src" else 1))
        changes = []
        for a in addresses:
            a = parse_address(a)
            m = ConjunctiveMatch(clause.rule_table, priority,
                                 [(address_match_key(a, addr_type == "src"), address_match_value(a))])
            ch = self._delete_conjunctive_match_flow(clause, m.key())
            if ch is not None:
                changes.append(ch)
        self._apply_changes(changes)

    def reassign_flow_priorities(self, updates: Dict[int, int], table: str):
        """ReassignFlowPriorities (network_policy.go:1746-1889), end state of the bundle."""
        add, dele = [], []
        moved = []
        for original, new in updates.items():
            for conj in self.policy_cache.with_priority(table, original):
                new_af = []
                for f in conj.action_flows:
                    if f.priority == original:
                        nf = f.copy_with_priority(new)
                        add.append(nf)
                        dele.append(f)
                        new_af.append(nf)
                    else:
                        new_af.append(f)
                for cl in conj.clauses():
                    for ctx in cl.matches.values():
                        if ctx.flow is not None:
                            add.append(ctx.flow.copy_with_priority(new))
                            dele.append(ctx.flow)
                moved.append((conj, new_af, new))
        # processFlowUpdates: an add that collides with a delete becomes a modify.
        add_ids = {flow_identity(f) for f in add}
        dele = [f for f in dele if flow_identity(f) not in add_ids]
        self._apply(add=add, delete=dele)
        for conj, new_af, new in moved:
            self.policy_cache.index(conj, False)
            conj.action_flows = new_af
            self.policy_cache.index(conj, True)
            for cl in conj.clauses():
                for ctx in list(cl.matches.values()):
                    self.global_cache.pop(ctx.match.key(), None)
                    if ctx.flow is not None:
                        ctx.flow = ctx.flow.copy_with_priority(new)
                    ctx.match.priority = new
                new_matches = {}
                for ctx in cl.matches.values():
                    new_matches[ctx.match.key()] = ctx
                    self.global_cache[ctx.match.key()] = ctx
                cl.matches = new_matches

    # ----- DNS packet-in conjunction (network_policy.go:697-789) ----------------------------
    def dns_packet_in_flow(self, cid) -> Flow:
        """pipeline.go:2080-2093: conj_id=id -> [meter,] paused packet-in to the FQDN controller, then
        IngressMetric."""
        acts = [("meter", PACKET_IN_METER_DNS)] if self.ovs_meters else []
        acts += [("controller", (PACKET_IN_CATEGORY_DNS,)), ("goto_table", "IngressMetric")]
        return Flow("AntreaPolicyIngressRule", PRIORITY_DNS_INTERCEPT, {"conj_id": (cid, None)}, acts, self.cookie)

    def new_dns_packet_in_conjunction(self, cid):
        """NewDNSPacketInConjunction (network_policy.go:697-779): service clause 1/2 = solicited DNS
        responses (ct_state=+rpl+trk, tcp/udp tp_src=53 per IP family), to clause 2/2 filled by
        AddAddressToDNSConjunction; no NetworkPolicyReference."""
        if cid in self.policy_cache:
            return
        table = "AntreaPolicyIngressRule"
        conj = Conjunction(cid)
        conj.np_ref = None
        conj.rule_table = table
        conj.action_flows = [self.dns_packet_in_flow(cid)]
        self._apply(add=conj.action_flows)
        conj.service_clause = Clause(ConjAction(cid, 1, 2), table, None)
        conj.to_clause = Clause(ConjAction(cid, 2, 2), table, None)
        ct = (MatchCTState, ("ctstate", 0b00101000, 0b00101000))
        changes = []
        for ipp in self.ip_protocols:
            tcp, udp = (MatchTCPSrcPort, MatchUDPSrcPort) if ipp == "ip" else (MatchTCPv6SrcPort, MatchUDPv6SrcPort)
            for key in (tcp, udp):
                m = ConjunctiveMatch(table, PRIORITY_DNS_INTERCEPT, [ct, (key, ("bitrange", DNS_PORT, None))])
                ch = self._add_conjunctive_match_flow(conj.service_clause, m, False, False)
                if ch is not None:
                    changes.append(ch)
        self._apply_changes(changes)
        self.policy_cache[cid] = conj

    def add_address_to_dns_conjunction(self, cid, addresses):
        """AddAddressToDNSConjunction (network_policy.go:781-784)."""
        self.add_policy_rule_address(cid, "dst", addresses, PRIORITY_DNS_INTERCEPT)

    def delete_address_from_dns_conjunction(self, cid, addresses):
        """DeleteAddressFromDNSConjunction (network_policy.go:786-789)."""
        self.delete_policy_rule_address(cid, "dst", addresses, PRIORITY_DNS_INTERCEPT)

    # ----- flow keys (network_policy.go:1520-1545, 1712-1736) ------------------------------
    def get_network_policy_flow_keys(self, name, namespace, policy_type) -> List[str]:
        """GetNetworkPolicyFlowKeys: per rule of the policy, action flows, conjunctive match flows,
        then drop flows (getAllFlowKeys); duplicates kept (shared contexts)."""
        keys = []
        for conj in self.policy_cache.values():
            if conj.np_ref is None:
                continue
            ptype, ns, pname = conj.np_ref[0], conj.np_ref[1], conj.np_ref[2]
            if (pname, ns, ptype) != (name, namespace, policy_type):
                continue
            fk, dk = [flow_dump_key(f) for f in conj.action_flows], []
            for cl in (conj.from_clause, conj.to_clause, conj.service_clause):
                if cl is None:
                    continue
                for ctx in cl.matches.values():
                    if ctx.flow is not None:
                        fk.append(flow_dump_key(ctx.flow))
                    if ctx.drop_flow is not None:
                        dk.append(flow_dump_key(ctx.drop_flow))
            keys += fk + dk
        return keys

    def get_policy_info_from_conjunction(self, rule_id):
        """GetPolicyInfoFromConjunction (network_policy.go:1555-1565)."""
        conj = self.policy_cache.get(rule_id)
        if conj is None or conj.np_ref is None:
            return (False, None, "", "", "")
        pr = conj.action_flow_priorities()
        if not pr:
            return (False, None, "", "", "")
        return (True, conj.np_ref, pr[0], conj.rule_name, conj.rule_log_label)


# ---------------------------------------------------------------------------------------------
# NetworkPolicyMetrics parsing (network_policy.go:1917-1980, 2034-2065)
# ---------------------------------------------------------------------------------------------
def parse_flow_to_map(flow: str) -> Dict[str, str]:
    out = {}
    for seg in flow.split(","):
        i = seg.find("=")
        if i == -1:
            continue
        k = seg[:i].strip()
        v = seg[i + 1:].strip()
        ai = v.find("actions")
        if ai != -1:
            v = v[:ai - 1]
        out[k] = v
    return out


def parse_metric_flow(fm: Dict[str, str]):
    pk = int(fm.get("n_packets", "0") or 0)
    by = int(fm.get("n_bytes", "0") or 0)
    if "reg0" in fm:
        return int(fm["reg3"], 0), (pk, by, pk)
    sessions = pk if "+" in fm.get("ct_state", "") else 0
    lab = fm["ct_label"]
    raw = lab[lab.index("0x") + 2: lab.index("/")]
    if len(raw) > 8:
        raw = raw[:len(raw) - 8]
    return int(raw, 16), (pk, by, sessions)


def network_policy_metrics(egress_dump: List[str], ingress_dump: List[str]):
    res = {}
    for dump in (egress_dump, ingress_dump):
        for f in dump:
            if "priority=%d," % PRIORITY_NORMAL not in f:
                continue
            rid, (p, b, s) = parse_metric_flow(parse_flow_to_map(f))
            if rid in res:
                op, ob, os_ = res[rid]
                res[rid] = (op + p, ob + b, os_ + s)
            else:
                res[rid] = (p, b, s)
    return res
