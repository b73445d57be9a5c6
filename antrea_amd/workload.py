"""Synthetic workloads for the BASELINE.json configs.

Rules are generated as the agent's reconciler would hand them to openflow.Client (table choice,
OF priorities from the priorityAssigner, ipBlock except-diffs), seeds as in the survey: rules
0xA1E47 (test/e2e/performance_test.go:36), packets 0xC1A55.

  C1  10 K8s NetworkPolicies x 3 rules over 100 local pods (10.10.0.0/24, ofports 3..102)
  C2  1k ACNP rules, tiers {50,100,150,200,250}; peers drawn from AddressGroups over 10k pod IPs
      (10.0.0.0/16); appliedTo = local ofports; 1-3 TCP ports per rule
  C3  100k ACNP/ANP rules = 50k ingress + 50k egress, 500 policies per direction x 100 rules
      (policy priority 1..100, unique OF priority per table); ipBlock peers with prefix U[8,32],
      20% with 1-3 excepts; TCP/UDP port ranges, start U[1,65535], width log-uniform 1..4096

Packet mix: each packet is aimed at a random rule r; 70% of addresses are drawn from
r's address space, the rest uniformly; 50% of ports fall inside r's port range; protocol TCP 70 /
UDP 25 / ICMP 5 unless the packet follows r's service; out_port (reg1) is the destination pod's
ofport.
"""
from __future__ import annotations

import ipaddress
import math
from typing import Dict, List

import numpy as np

from . import caller

RULE_SEED = 0xA1E47
PKT_SEED = 0xC1A55
TIERS = [50, 100, 150, 200, 250]


def _pods(n, base):
    b = int(ipaddress.ip_address(base))
    ips = [b + 1 + i for i in range(n)]
    return np.array(ips, dtype=np.uint32), np.arange(3, 3 + n, dtype=np.uint32)


def _ip(v):
    return str(ipaddress.ip_address(int(v)))


class Workload:
    """rules (gpc rule dicts) + the arrays the packet generator needs."""

    def __init__(self, name):
        self.name = name
        self.rules: List[dict] = []
        self.local_ips = np.zeros(0, np.uint32)
        self.local_ports = np.zeros(0, np.uint32)
        # per-rule packet-generation metadata (numpy, len = n_rules)
        self.meta = {}

    @property
    def n_rules(self):
        return len(self.rules)


def _assign_priorities(specs, baseline=False):
    """specs: list of (tier, policy_prio, rule_prio) per rule of ONE table -> OF priorities."""
    pa = caller.PriorityAssigner(is_baseline=baseline)
    pa.register_priorities(list(specs))
    return [pa.get_of_priority(p)[0] for p in specs]


# ------------------------------------------------------------------------------------- C1
def config1(seed=RULE_SEED) -> Workload:
    rng = np.random.default_rng(seed)
    wl = Workload("C1")
    wl.local_ips, wl.local_ports = _pods(100, "10.10.0.0")
    fid = 1
    m = {k: [] for k in ("dir", "src_base", "src_len", "dst_base", "dst_len", "ports", "proto", "plo", "phi")}
    for np_i in range(10):
        applied = rng.choice(100, size=rng.integers(5, 20), replace=False)
        for r_i in range(3):
            peers = rng.choice(100, size=rng.integers(1, 10), replace=False)
            svc = None
            plo = phi = 0
            proto = 6
            if rng.random() < 0.7:
                port = int(rng.choice([80, 443, 8080, 53, 5432]))
                proto = 6 if port != 53 else 17
                svc = [{"protocol": "TCP" if proto == 6 else "UDP", "port": port}]
                plo = phi = port
            direction = "In" if r_i < 2 else "Out"
            ref = {"policy_type": "K8sNetworkPolicy", "policy_namespace": "ns%d" % np_i, "policy_name": "np%d" % np_i,
                   "policy_uid": "uid-%d" % np_i, "name": "rule%d" % r_i, "flow_id": fid}
            if direction == "In":
                frm = [_ip(wl.local_ips[p]) for p in peers]
                if rng.random() < 0.3:
                    frm += [{"ipnet": "172.16.%d.0/24" % rng.integers(0, 255)}]
                rule = dict(ref, direction="In", table="IngressRule", **{"from": frm},
                            to=[{"ofport": int(wl.local_ports[a])} for a in applied], service=svc)
            else:
                to = [_ip(wl.local_ips[p]) for p in peers]
                rule = dict(ref, direction="Out", table="EgressRule", **{"from": [_ip(wl.local_ips[a]) for a in applied]},
                            to=to, service=svc)
            wl.rules.append(rule)
            m["dir"].append(0 if direction == "In" else 1)
            m["src_base"].append(int(wl.local_ips[peers[0]] if direction == "In" else wl.local_ips[applied[0]]))
            m["src_len"].append(32)
            m["dst_base"].append(int(wl.local_ips[applied[0]] if direction == "In" else wl.local_ips[peers[0]]))
            m["dst_len"].append(32)
            m["ports"].append(int(wl.local_ports[applied[0]] if direction == "In" else wl.local_ports[peers[0]]))
            m["proto"].append(proto)
            m["plo"].append(plo)
            m["phi"].append(phi)
            fid += 1
    wl.meta = {k: np.array(v) for k, v in m.items()}
    return wl


# ------------------------------------------------------------------------------------- C2 / C3
def _acnp_config(name, n_policies_per_dir, rules_per_policy, peer_fn, svc_fn, seed, n_local=100,
                 local_base="10.0.0.0", actions=(0.6, 0.3, 0.1)) -> Workload:
    rng = np.random.default_rng(seed)
    wl = Workload(name)
    wl.local_ips, wl.local_ports = _pods(n_local, local_base)
    m = {k: [] for k in ("dir", "src_base", "src_len", "dst_base", "dst_len", "ports", "proto", "plo", "phi")}
    fid = 1
    for direction, table in (("In", "AntreaPolicyIngressRule"), ("Out", "AntreaPolicyEgressRule")):
        specs, pending = [], []
        for pi in range(n_policies_per_dir):
            tier = TIERS[pi % len(TIERS)]
            ppri = float(1 + (pi // len(TIERS)) % 100)
            applied = rng.choice(n_local, size=int(rng.integers(1, 11)), replace=False)
            ptype = "AntreaClusterNetworkPolicy" if pi % 4 else "AdminNetworkPolicy"
            for ri in range(rules_per_policy):
                peers, (pbase, plen) = peer_fn(rng)
                svc, proto, plo, phi = svc_fn(rng)
                u = rng.random()
                action = "Allow" if u < actions[0] else ("Drop" if u < actions[0] + actions[1] else "Pass")
                rule = {"direction": direction, "table": table, "action": action, "flow_id": fid,
                        "policy_type": ptype, "policy_namespace": "", "policy_name": "%s-%s-%d" % (name, direction, pi),
                        "policy_uid": "uid-%s-%d" % (direction, pi), "name": "rule-%d" % ri, "tier_priority": tier,
                        "service": svc}
                if direction == "In":
                    rule["from"] = peers
                    rule["to"] = [{"ofport": int(wl.local_ports[a])} for a in applied]
                else:
                    rule["from"] = [_ip(wl.local_ips[a]) for a in applied]
                    rule["to"] = peers
                specs.append((tier, ppri, ri))
                pending.append(rule)
                a0 = applied[0]
                m["dir"].append(0 if direction == "In" else 1)
                if direction == "In":
                    m["src_base"].append(pbase)
                    m["src_len"].append(plen)
                    m["dst_base"].append(int(wl.local_ips[a0]))
                    m["dst_len"].append(32)
                    m["ports"].append(int(wl.local_ports[a0]))
                else:
                    m["src_base"].append(int(wl.local_ips[a0]))
                    m["src_len"].append(32)
                    m["dst_base"].append(pbase)
                    m["dst_len"].append(plen)
                    m["ports"].append(int(wl.local_ports[rng.integers(0, n_local)]))
                m["proto"].append(proto)
                m["plo"].append(plo)
                m["phi"].append(phi)
                fid += 1
        prios = _assign_priorities(specs)
        for rule, p in zip(pending, prios):
            rule["priority"] = int(p)
        wl.rules.extend(pending)
    wl.meta = {k: np.array(v) for k, v in m.items()}
    return wl


def config2(seed=RULE_SEED) -> Workload:
    """1k ACNP rules: 50 policies per direction x 10 rules; peers = address-group pod IPs."""
    group_pool = np.arange(10000, dtype=np.uint32) + np.uint32(int(ipaddress.ip_address("10.0.100.0")))
    rng0 = np.random.default_rng(seed + 1)
    groups = [rng0.choice(group_pool, size=int(rng0.integers(50, 1000)), replace=False) for _ in range(64)]

    def peers(rng):
        g = groups[int(rng.integers(0, len(groups)))]
        return [_ip(v) for v in g], (int(g[0]), 32)

    def svc(rng):
        ports = rng.choice([80, 443, 8080, 8443, 3306, 5432, 6379, 9090], size=int(rng.integers(1, 4)), replace=False)
        return [{"protocol": "TCP", "port": int(p)} for p in ports], 6, int(ports[0]), int(ports[0])

    return _acnp_config("C2", 50, 10, peers, svc, seed)


def config2g(seed=RULE_SEED, n_groups=16, group_size=10000) -> Workload:
    """C2 at the stated group size (BASELINE configs[1]: "AddressGroups of 10k pod IPs"): the same
    1k ACNP rules over 5 tiers, but every rule's From is one of `n_groups` AddressGroups of
    `group_size` Pod IPs drawn from the 10.0.0.0/16 Pods (10M address atoms in all). Packets: 70% of
    sources from the /16 (a Pod of the cluster, in the rule's group about 15% of the time)."""
    pool = np.arange(1, 65535, dtype=np.uint32) + np.uint32(int(ipaddress.ip_address("10.0.0.0")))
    rng0 = np.random.default_rng(seed + 2)
    groups = [[_ip(v) for v in np.sort(rng0.choice(pool, size=group_size, replace=False))] for _ in range(n_groups)]

    def peers(rng):
        return groups[int(rng.integers(0, n_groups))], (int(pool[0]) & 0xFFFF0000, 16)

    def svc(rng):
        ports = rng.choice([80, 443, 8080, 8443, 3306, 5432, 6379, 9090], size=int(rng.integers(1, 4)), replace=False)
        return [{"protocol": "TCP", "port": int(p)} for p in ports], 6, int(ports[0]), int(ports[0])

    return _acnp_config("C2g", 50, 10, peers, svc, seed, local_base="10.1.0.0")


def _rand_block(rng):
    plen = int(rng.integers(8, 33))
    base = int(rng.integers(0, 1 << 32)) & (((1 << plen) - 1) << (32 - plen)) if plen else 0
    block = {"cidr": "%s/%d" % (_ip(base), plen)}
    if plen < 32 and rng.random() < 0.2:
        exc = []
        for _ in range(int(rng.integers(1, 4))):
            el = int(rng.integers(plen + 1, 33))
            eb = (base | (int(rng.integers(0, 1 << 32)) & ((1 << (32 - plen)) - 1))) & (((1 << el) - 1) << (32 - el))
            exc.append("%s/%d" % (_ip(eb), el))
        block["except"] = exc
    return block, base, plen


def config3(seed=RULE_SEED, n_policies_per_dir=500, rules_per_policy=100) -> Workload:
    """100k rules (50k per direction) with ipBlock CIDRs and L4 port ranges."""

    def peers(rng):
        block, base, plen = _rand_block(rng)
        return caller.ip_blocks_to_of_addresses([block]), (base, plen)

    def svc(rng):
        proto = "TCP" if rng.random() < 0.5 else "UDP"
        start = int(rng.integers(1, 65536))
        width = int(round(math.exp(rng.uniform(0, math.log(4096)))))
        end = min(65535, start + width - 1)
        s = {"protocol": proto, "port": start}
        if end > start:
            s["end_port"] = end
        return [s], 6 if proto == "TCP" else 17, start, end

    return _acnp_config("C3", n_policies_per_dir, rules_per_policy, peers, svc, seed)


# ------------------------------------------------------------------------------ AntreaProxy (C4)
SVC_PROTOS = (("TCP", 6), ("UDP", 17), ("SCTP", 132))


NODE_PORT_ADDRESSES = ("192.168.77.100", "192.168.77.101")  # the Node's NodePort addresses (nodeport_frac > 0)
VIRTUAL_NODE_PORT_DNAT = "169.254.0.252"                    # config.VirtualNodePortDNATIPv4


def add_services(wl: Workload, n_services: int, eps_per_service: int, seed=RULE_SEED + 4, remote_frac=0.7,
                 noep_frac=0.02, local_policy_frac=0.1, svc_frac=0.5, nodeport_frac=0.0) -> Workload:
    """ClusterIP Services (10.96.0.0/12) with `eps_per_service` Endpoints each: local Endpoints are
    the workload's local Pods (ofports known to the Pod map), remote ones are Pods on other Nodes
    (10.128.0.0/9). A fraction of Services has no Endpoints, a fraction Local traffic policy.
    `svc_frac` of the generated packets are aimed at a Service (ip, port, protocol).
    `nodeport_frac` > 0: that fraction are NodePort Services (installed with the virtual NodePort
    DNAT IP, as the proxier does, on ports 30000-32767 unique per protocol); their packets go to one
    of NODE_PORT_ADDRESSES or the virtual IP; wl.node_port_addresses is set."""
    rng = np.random.default_rng(seed)
    base = int(ipaddress.ip_address("10.96.0.0"))
    ips = base + 1 + rng.choice(1 << 20, size=n_services, replace=False)
    ports = rng.integers(1, 65536, size=n_services)
    pk = rng.choice(3, size=n_services, p=[0.8, 0.15, 0.05])
    wl.services, wl.groups, wl.endpoint_flows = [], {}, []
    wl.pods = {int(ip): int(port) for ip, port in zip(wl.local_ips, wl.local_ports)}
    for i in range(n_services):
        proto = SVC_PROTOS[pk[i]][0]
        n_ep = 0 if rng.random() < noep_frac else eps_per_service
        eps = []
        for _ in range(n_ep):
            if rng.random() < remote_frac:
                ip = int(ipaddress.ip_address("10.128.0.0")) + int(rng.integers(1, 1 << 23))
                eps.append({"ip": _ip(ip), "port": int(rng.integers(1024, 65536)), "is_local": False,
                            "node_name": "node%d" % int(rng.integers(1, 64))})
            else:
                j = int(rng.integers(0, len(wl.local_ips)))
                eps.append({"ip": _ip(wl.local_ips[j]), "port": int(rng.integers(1024, 65536)), "is_local": True,
                            "node_name": "node0"})
        local = rng.random() < local_policy_frac
        cgid, lgid = 2 * i + 1, 2 * i + 2
        wl.groups[lgid if local else cgid] = eps
        if eps:
            wl.endpoint_flows.append((proto, eps))
        wl.services.append({"ip": _ip(ips[i]), "port": int(ports[i]), "protocol": proto, "cluster_group_id": cgid,
                            "local_group_id": lgid, "traffic_policy_local": bool(local)})
    if nodeport_frac > 0:  # (drawn after the ClusterIP set: other workloads keep their streams)
        nrng = np.random.default_rng(seed + 17)
        addrs = [int(ipaddress.ip_address(a)) for a in NODE_PORT_ADDRESSES + (VIRTUAL_NODE_PORT_DNAT,)]
        taken = set()
        for i in np.nonzero(nrng.random(n_services) < nodeport_frac)[0]:
            s = wl.services[i]
            while True:
                port = int(nrng.integers(30000, 32768))
                if (s["protocol"], port) not in taken:
                    break
            taken.add((s["protocol"], port))
            if s["traffic_policy_local"] and s["local_group_id"] in wl.groups:  # (external + Local: not modelled)
                wl.groups[s["cluster_group_id"]] = wl.groups.pop(s["local_group_id"])
            s.update(ip=VIRTUAL_NODE_PORT_DNAT, port=port, is_nodeport=True, is_external=True, traffic_policy_local=False)
            ips[i] = addrs[int(nrng.integers(len(addrs)))]  # the packets' destination
            ports[i] = port
        wl.node_port_addresses = list(NODE_PORT_ADDRESSES)
    wl.svc_meta = {"ip": ips.astype(np.uint32), "port": ports.astype(np.uint16),
                   "proto": np.array([SVC_PROTOS[k][1] for k in pk], np.uint8)}
    wl.svc_frac = svc_frac
    return wl


def install_services(clf, wl: Workload):
    """The AntreaProxy calls for wl's Services (client.go:710-815 order: groups, Endpoint flows,
    Service flows) plus the Pod map."""
    for ip, port in wl.pods.items():
        clf.install_pod(_ip(ip), port)
    if getattr(wl, "node_port_addresses", None):
        clf.set_node_port_addresses(wl.node_port_addresses)
    for gid, eps in wl.groups.items():
        clf.install_service_group(gid, eps)
    for proto, eps in wl.endpoint_flows:
        clf.install_endpoint_flows(proto, eps)
    for cfg in wl.services:
        clf.install_service_flows(cfg)


def config4(seed=RULE_SEED) -> Workload:
    """C3 + 10k Services x 10 Endpoints (AntreaProxy ServiceLB / EndpointDNAT in front of policy)."""
    return add_services(config3(seed), 10000, 10)


CONFIGS = {"C1": config1, "C2": config2, "C2g": config2g, "C3": config3, "C4": config4}


# ------------------------------------------------------------------------------------- packets
def gen_packets(wl: Workload, n: int, seed=PKT_SEED) -> Dict[str, np.ndarray]:
    """SoA packet columns (numpy) for workload `wl` (see module docstring for the mix)."""
    rng = np.random.default_rng(seed)
    m = wl.meta
    nr = len(m["dir"])
    r = rng.integers(0, nr, size=n)

    def in_prefix(base, plen):
        plen = plen.astype(np.int64)
        host_bits = (32 - plen).astype(np.uint64)
        rnd = rng.integers(0, 1 << 32, size=len(base), dtype=np.uint64)
        mask = ((np.uint64(1) << host_bits) - np.uint64(1))
        return ((base.astype(np.uint64) & ~mask & np.uint64(0xFFFFFFFF)) | (rnd & mask)).astype(np.uint32)

    uni = lambda: rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    src = np.where(rng.random(n) < 0.7, in_prefix(m["src_base"][r], m["src_len"][r]), uni())
    dst = np.where(rng.random(n) < 0.7, in_prefix(m["dst_base"][r], m["dst_len"][r]), uni())
    nl = len(wl.local_ports)
    rand_local = rng.integers(0, nl, size=n)
    out_port = np.where(rng.random(n) < 0.7, m["ports"][r], wl.local_ports[rand_local]).astype(np.uint32)
    follow = rng.random(n) < 0.7
    u = rng.random(n)
    mix_proto = np.where(u < 0.70, 6, np.where(u < 0.95, 17, 1)).astype(np.uint8)
    proto = np.where(follow, m["proto"][r], mix_proto).astype(np.uint8)
    plo, phi = m["plo"][r], m["phi"][r]
    width = np.maximum(phi - plo + 1, 1)
    inside = (plo + (rng.random(n) * width).astype(np.int64)).clip(0, 65535)
    dport = np.where((rng.random(n) < 0.5) & (plo > 0), inside, rng.integers(1, 65536, size=n)).astype(np.uint16)
    sport = rng.integers(1024, 65536, size=n).astype(np.uint16)
    icmp = proto == 1
    sport = np.where(icmp, rng.choice([0, 3, 8, 11], size=n), sport).astype(np.uint16)
    dport = np.where(icmp, 0, dport).astype(np.uint16)
    length = rng.integers(64, 1500, size=n).astype(np.uint16)
    if getattr(wl, "svc_meta", None) is not None:  # aim svc_frac of the packets at a Service
        sm = wl.svc_meta
        k = rng.integers(0, len(sm["ip"]), size=n)
        to_svc = rng.random(n) < wl.svc_frac
        dst = np.where(to_svc, sm["ip"][k], dst).astype(np.uint32)
        dport = np.where(to_svc, sm["port"][k], dport).astype(np.uint16)
        proto = np.where(to_svc, sm["proto"][k], proto).astype(np.uint8)
        sport = np.where(to_svc, rng.integers(1024, 65536, size=n), sport).astype(np.uint16)
    return {"src": src, "dst": dst, "sport": sport, "dport": dport, "proto": proto, "out_port": out_port,
            "len": length}


def gen_packets_torch(wl: Workload, n: int, seed=PKT_SEED, device="cuda"):
    """Same mix as gen_packets, generated directly in device memory (bench: 64M packets/GPU)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    m = {k: torch.as_tensor(np.asarray(v, dtype=np.int64), device=device) for k, v in wl.meta.items()}
    nr = len(wl.meta["dir"])
    r = torch.randint(0, nr, (n,), generator=g, device=device)

    def rnd32():
        return torch.randint(0, 1 << 32, (n,), generator=g, device=device, dtype=torch.int64)

    def frac():
        return torch.rand(n, generator=g, device=device)

    def in_prefix(base, plen):
        hostmask = (torch.ones_like(plen) << (32 - plen)) - 1
        return ((base & ~hostmask) | (rnd32() & hostmask)) & 0xFFFFFFFF

    src = torch.where(frac() < 0.7, in_prefix(m["src_base"][r], m["src_len"][r]), rnd32())
    dst = torch.where(frac() < 0.7, in_prefix(m["dst_base"][r], m["dst_len"][r]), rnd32())
    local_ports = torch.as_tensor(wl.local_ports.astype(np.int64), device=device)
    rl = torch.randint(0, len(wl.local_ports), (n,), generator=g, device=device)
    out_port = torch.where(frac() < 0.7, m["ports"][r], local_ports[rl])
    u = frac()
    mix = torch.where(u < 0.70, 6, torch.where(u < 0.95, 17, 1))
    proto = torch.where(frac() < 0.7, m["proto"][r], mix)
    plo, phi = m["plo"][r], m["phi"][r]
    width = torch.clamp(phi - plo + 1, min=1)
    inside = torch.clamp(plo + (frac() * width).long(), 0, 65535)
    dport = torch.where((frac() < 0.5) & (plo > 0), inside, torch.randint(1, 65536, (n,), generator=g, device=device))
    sport = torch.randint(1024, 65536, (n,), generator=g, device=device)
    icmp = proto == 1
    types = torch.tensor([0, 3, 8, 11], device=device)[torch.randint(0, 4, (n,), generator=g, device=device)]
    sport = torch.where(icmp, types, sport)
    dport = torch.where(icmp, torch.zeros_like(dport), dport)
    length = torch.randint(64, 1500, (n,), generator=g, device=device)
    if getattr(wl, "svc_meta", None) is not None:
        sm = {k: torch.as_tensor(v.astype(np.int64), device=device) for k, v in wl.svc_meta.items()}
        k = torch.randint(0, len(wl.svc_meta["ip"]), (n,), generator=g, device=device)
        to_svc = frac() < wl.svc_frac
        dst = torch.where(to_svc, sm["ip"][k], dst)
        dport = torch.where(to_svc, sm["port"][k], dport)
        proto = torch.where(to_svc, sm["proto"][k], proto)
    u32 = lambda t: (t & 0xFFFFFFFF).to(torch.int64).to(torch.uint32) if hasattr(torch, "uint32") else t.to(torch.int32)
    return {"src": u32(src), "dst": u32(dst), "sport": sport.to(torch.int16), "dport": dport.to(torch.int16),
            "proto": proto.to(torch.uint8), "out_port": u32(out_port), "len": length.to(torch.int16)}


# ------------------------------------------------------------------------------------- IPv6
# IPv6 (and dual-stack) variants: every IPv4 address / CIDR of a workload embedded in fd00:10::/96
# (a.b.c.d -> fd00:10::a.b.c.d, /L -> /(96 + L)). The rule structure, priorities and conj ids are
# unchanged, so IPv6 packets mapped the same way must get exactly the IPv4 verdicts (metamorphic
# parity of the IPv6 image against the IPv4 one, itself pinned by the oracles).
V6_EMBED = int(ipaddress.IPv6Address("fd00:10::"))
_V6_PREFIX12 = np.frombuffer(V6_EMBED.to_bytes(16, "big")[:12], dtype=np.uint8)


# Embeddings of the IPv4 workloads in IPv6, both prefix-preserving for IPv4 prefixes of length >= 2
# (a in P <=> emb(a) in emb(P)), so the IPv4 oracle's verdicts apply to the embedded packets:
#   "96"      a -> fd00:10::a (one /96; an IPv4 /L is an IPv6 /96+L)
#   "multi48" the top 2 bits of a pick one of four /48s fd00:0:k::/48, the other 30 bits follow the
#             /48 (an IPv4 /L is an IPv6 /46+L): rule sets spread over several /48s
V6_MULTI48 = int(ipaddress.IPv6Address("fd00::"))


def v6_embed(v4: int, embed: str = "96") -> int:
    if embed == "96":
        return V6_EMBED | v4
    return V6_MULTI48 | ((v4 >> 30) << 80) | ((v4 & 0x3FFFFFFF) << 50)


def v6_embed_len(plen: int, embed: str = "96") -> int:
    if embed == "96":
        return 96 + plen
    if plen < 2:
        raise ValueError("multi48 embeds IPv4 prefixes of length >= 2 only")
    return 46 + plen


def _v6_addr(a, embed="96"):
    if isinstance(a, str):
        if "." not in a:
            return a
        if "/" in a:
            return _v6_addr({"ipnet": a}, embed)["ipnet"]
        return str(ipaddress.IPv6Address(v6_embed(int(ipaddress.ip_address(a)), embed)))
    (k, v), = a.items()
    if k in ("ip", "ctip"):
        return {k: str(ipaddress.IPv6Address(v6_embed(int(ipaddress.ip_address(v)), embed)))}
    if k in ("ipnet", "ctipnet"):
        n = ipaddress.ip_network(v, strict=False)
        return {k: "%s/%d" % (ipaddress.IPv6Address(v6_embed(int(n.network_address), embed)),
                              v6_embed_len(n.prefixlen, embed))}
    return a


def to_ipv6(wl: Workload, dual=False, embed="96") -> Workload:
    """The workload with its addresses in IPv6 (dual=True: both families in every peer list)."""
    import copy
    out = Workload(wl.name + ("dual" if dual else "v6"))
    out.local_ips, out.local_ports, out.meta = wl.local_ips, wl.local_ports, wl.meta
    for r in wl.rules:
        r6 = copy.deepcopy(r)
        for side in ("from", "to"):
            if r.get(side) is not None:
                mapped = [_v6_addr(a, embed) for a in r[side]]
                r6[side] = (list(r[side]) + [m for m, a in zip(mapped, r[side]) if m != a]) if dual else mapped
        out.rules.append(r6)
    return out


def v6_bytes(v4: np.ndarray, embed="96") -> np.ndarray:
    """(n,) IPv4 addresses -> (n, 16) uint8 network-order IPv6 addresses (the embedding above)."""
    v4 = np.asarray(v4, dtype=np.uint32)
    if embed == "96":
        tail = v4.astype(">u4").view(np.uint8).reshape(-1, 4)
        return np.ascontiguousarray(np.concatenate([np.broadcast_to(_V6_PREFIX12, (len(v4), 12)), tail], axis=1))
    return np.array([list(v6_embed(int(a), embed).to_bytes(16, "big")) for a in v4], dtype=np.uint8).reshape(-1, 16)


def packets_to_v6(cols: Dict[str, np.ndarray], embed="96") -> Dict[str, np.ndarray]:
    """IPv4 packet columns -> the IPv6 batch of the same packets (ICMP -> ICMPv6)."""
    out = {k: v for k, v in cols.items() if k not in ("src", "dst", "ct_src", "ct_dst")}
    for k in ("src", "dst", "ct_src", "ct_dst"):
        if k in cols:
            out[k + "6"] = v6_bytes(cols[k], embed)
    out["proto"] = np.where(cols["proto"] == 1, 58, cols["proto"]).astype(np.uint8)
    return out


def packets_to_v6_torch(cols, embed="96"):
    """Device version of packets_to_v6 (bench): (n, 16) uint8 address columns (the embedding above)."""
    import torch
    out = {k: v for k, v in cols.items() if k not in ("src", "dst", "ct_src", "ct_dst")}
    be32 = lambda x: torch.stack([(x >> 24) & 255, (x >> 16) & 255, (x >> 8) & 255, x & 255], dim=1)
    for k in ("src", "dst", "ct_src", "ct_dst"):
        if k not in cols:
            continue
        v = cols[k].to(torch.int64) & 0xFFFFFFFF
        n = v.shape[0]
        if embed == "96":
            head = torch.as_tensor(_V6_PREFIX12.copy(), device=v.device).expand(n, 12)
            out[k + "6"] = torch.cat([head, be32(v).to(torch.uint8)], dim=1).contiguous()
            continue
        # multi48: fd00:0:k::/48 (k = top 2 bits), then the other 30 bits at bits 79..50
        z = torch.zeros((n, 16), dtype=torch.int64, device=v.device)
        z[:, 0] = 0xFD
        z[:, 5] = v >> 30
        z[:, 6:10] = be32(((v & 0x3FFFFFFF) << 2) & 0xFFFFFFFF)
        out[k + "6"] = z.to(torch.uint8).contiguous()
    p = cols["proto"]
    out["proto"] = torch.where(p == 1, torch.full_like(p, 58), p)
    return out
