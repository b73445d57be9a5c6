"""Parser for the ovs-ofctl flow text Antrea emits (TEST INFRASTRUCTURE ONLY).

The format is the one produced by `FlowModToString` (`pkg/ovs/openflow/utils.go:1222-1241`) and by
`ovs-ofctl dump-flows` (as parsed by `parseFlowToMap`, `pkg/agent/openflow/network_policy.go:1948`).
A parsed flow is a dict:
    {"table": str, "priority": int, "match": {field: (value, mask)}, "actions": [tuple, ...],
     "n_packets": int, "n_bytes": int}
Field values are integers; masks are integers (None = exact). Prefix fields are converted to masks.
"""
from __future__ import annotations

import ipaddress
import re

PROTO_WORDS = {
    "ip": (0x0800, None), "ipv6": (0x86DD, None), "arp": (0x0806, None),
    "tcp": (0x0800, 6), "tcp6": (0x86DD, 6), "udp": (0x0800, 17), "udp6": (0x86DD, 17),
    "sctp": (0x0800, 132), "sctp6": (0x86DD, 132), "icmp": (0x0800, 1), "icmp6": (0x86DD, 58),
    "igmp": (0x0800, 2),
}
CT_BITS = {"new": 0, "est": 1, "rel": 2, "rpl": 3, "inv": 4, "trk": 5, "snat": 6, "dnat": 7}


def _split_top(s: str, sep: str = ","):
    """Split on `sep` at parenthesis depth 0."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return out


def _num(s):
    return int(s, 0)


def _vm(s):
    if "/" in s:
        v, m = s.split("/", 1)
        return _num(v), _num(m)
    return _num(s), None


def _ip(s, bits):
    if "/" in s:
        a, p = s.split("/", 1)
        ip = int(ipaddress.ip_address(a))
        plen = int(p)
        mask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1) if plen else 0
        return ip & mask, mask
    return int(ipaddress.ip_address(s)), None


def parse_actions(s: str):
    acts = []
    for a in _split_top(s):
        a = a.strip()
        if not a:
            continue
        if a == "drop":
            acts.append(("drop",))
        elif a.startswith("conjunction("):
            m = re.match(r"conjunction\((\d+),(\d+)/(\d+)\)", a)
            acts.append(("conjunction", int(m.group(1)), int(m.group(2)), int(m.group(3))))
        elif a.startswith("set_field:"):
            body, dst = a[len("set_field:"):].split("->")
            v, m = _vm(body)
            if dst == "ct_label":
                acts.append(("set_ct_label", v, m))
            else:
                acts.append(("set_reg", int(dst[3:]), v, m))
        elif a.startswith("ct("):
            inner = a[3:-1]
            table, labels, nat = None, [], None
            for part in _split_top(inner):
                if part.startswith("table="):
                    table = part[6:]
                elif part.startswith("nat(dst=") and part.endswith(")"):
                    ip, _, port = part[len("nat(dst="):-1].rpartition(":")
                    nat = (int(ipaddress.ip_address(ip)), int(port))
                elif part.startswith("exec("):
                    for ea in _split_top(part[5:-1]):
                        if ea.startswith("set_field:") and ea.endswith("->ct_label"):
                            v, m = _vm(ea[len("set_field:"):-len("->ct_label")])
                            labels.append((v, m))
            acts.append(("ct_commit", table, labels, nat))
        elif a.startswith("goto_table:"):
            acts.append(("goto_table", a[len("goto_table:"):]))
        elif a.startswith("resubmit(,") or a.startswith("resubmit:"):
            t = a[len("resubmit(,"):-1] if a.startswith("resubmit(,") else a[len("resubmit:"):]
            acts.append(("goto_table", t))
        elif a.startswith("group:"):
            acts.append(("group", int(a[6:])))
        elif a.startswith("meter:"):
            acts.append(("meter", int(a[6:])))
        elif a.startswith("controller(") and a.endswith(")"):
            kv = dict(x.split("=", 1) for x in _split_top(a[len("controller("):-1]) if "=" in x)
            ud = tuple(int(b, 16) for b in kv["userdata"].split(".")) if "userdata" in kv else ()
            acts.append(("controller", ud))
        else:
            acts.append(("other", a))
    return acts


def parse_group(line: str) -> dict:
    """`group_id=G,type=select,bucket=bucket_id:B,weight:W,actions=...,bucket=...` (the text the
    reference tests print for a binding.Group, client_test.go:1024-1090)."""
    head, *buckets = line.strip().split(",bucket=")
    gid = int(head.split(",")[0].split("=")[1])
    out = {"id": gid, "buckets": []}
    for b in buckets:
        meta, _, acts = b.partition(",actions=")
        kv = dict(x.split(":", 1) for x in meta.split(","))
        out["buckets"].append({"id": int(kv["bucket_id"]), "weight": int(kv["weight"]),
                               "actions": parse_actions(acts)})
    return out


def parse_flow(line: str) -> dict:
    line = line.strip()
    head, _, actstr = line.partition(" actions=")
    flow = {"table": None, "priority": 32768, "match": {}, "actions": parse_actions(actstr),
            "n_packets": 0, "n_bytes": 0, "cookie": 0}
    m = flow["match"]
    for tok in [t.strip() for t in head.replace(", ", ",").split(",")]:
        if not tok:
            continue
        if "=" not in tok:
            eth, proto = PROTO_WORDS[tok]
            m["dl_type"] = (eth, None)
            if proto is not None:
                m["nw_proto"] = (proto, None)
            continue
        k, v = tok.split("=", 1)
        if k == "table":
            flow["table"] = v
        elif k == "priority":
            flow["priority"] = int(v)
        elif k == "cookie":
            flow["cookie"] = _num(v.split("/")[0])
        elif k in ("n_packets", "n_bytes"):
            flow[k] = int(v)
        elif k in ("duration", "idle_timeout", "hard_timeout", "idle_age", "hard_age"):
            continue
        elif k == "conj_id":
            m["conj_id"] = (int(v), None)
        elif k == "ct_state":
            data = mask = 0
            for sign, name in re.findall(r"([+-])([a-z]+)", v):
                b = 1 << CT_BITS[name]
                mask |= b
                if sign == "+":
                    data |= b
            m["ct_state"] = (data, mask)
        elif k in ("ct_label", "ct_mark"):
            m[k] = _vm(v)
        elif k in ("nw_src", "nw_dst", "ct_nw_src", "ct_nw_dst"):
            m[k] = _ip(v, 32)
        elif k in ("ipv6_src", "ipv6_dst", "ct_ipv6_src", "ct_ipv6_dst"):
            m[k] = _ip(v, 128)
        elif re.fullmatch(r"reg\d+", k):
            m[k] = _vm(v)
        elif k in ("tun_id", "in_port", "icmp_type", "icmp_code", "icmpv6_type", "icmpv6_code"):
            m[k.replace("icmpv6", "icmp")] = _vm(v)
        elif k in ("tp_src", "tp_dst"):
            m[k] = _vm(v)
        else:
            raise ValueError("unsupported match field %r in %r" % (k, line))
    return flow
