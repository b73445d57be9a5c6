"""CPU restatement of AntreaProxy's flow side -- TEST INFRASTRUCTURE (checker only; the product's
Service stage is antrea_amd/csrc/service.cpp + core.hpp lb_stage).

What the agent's openflow client installs for a ClusterIP Service, as flow / group text in the
reference's dump format (`pkg/ovs/openflow/utils.go` FlowModToString, as the goldens of
`client_test.go:1025-1279` print it):

* `serviceEndpointGroup` (`pkg/agent/openflow/pipeline.go:2553-2592`) via `InstallServiceGroup`
  (`client.go:710-727`): a select group with one weight-100 bucket per Endpoint loading the
  Endpoint IP (reg3) and port (reg4[0..15]), RemoteEndpointRegMark (reg4[26]) for remote
  non-hostNetwork Endpoints, then resubmit to EndpointDNAT (ServiceLB with session affinity); no
  Endpoints: one bucket loading SvcNoEpRegMark (reg0[14]).
* `endpointDNATFlow` (`pipeline.go:2502-2528`) and, for local Endpoints, `podHairpinSNATFlow`
  (`:3052-3065`) via `InstallEndpointFlows` (`client.go:750-770`, cache key
  `generateEndpointFlowCacheKey` `:742`).
* `serviceLBFlows` (`pipeline.go:2374-2431`) via `InstallServiceFlows` (`client.go:790-807`, cache
  key `generateServicePortFlowCacheKey` `:746`): one flow at priority 200 matching
  EpToSelectRegMark + Service IP / protocol / port, loading RewriteMACRegMark, EpSelectedRegMark and
  (AntreaPolicy on) ServiceGroupIDField = the group it selects, then `group:`.

* `nodePortMarkFlows` (`pipeline.go:2282-2314`, proxyAll): ToNodePortAddressRegMark (reg4[19]) for
  packets to a NodePort address or the virtual NodePort DNAT IP; a NodePort Service's ServiceLB
  flow matches that mark and the port instead of the Service IP (`:2381-2387`).

Only the shapes the product's data path takes are restated (IPv4; no session affinity learn flow,
DSR, nested Services, nor the short-circuit flow of external Local Services): the others are
rejected by both sides. Pinned by the
Service goldens of `client_test.go` (tests/golden/service_flows.json, tests/test_service.py).
"""
from __future__ import annotations

import ipaddress
from typing import Dict, List

SERVICE_COOKIE = 0x1030000000000  # cookie allocator round 1, category Service (as the goldens print it)
PRIORITY_NORMAL, PRIORITY_LOW = 200, 190
PROTOCOLS = {"TCP": "tcp", "UDP": "udp", "SCTP": "sctp"}  # binding.Protocol names, IPv4 (utils.go:298-354)
DNAT_CT_ZONE = 65520                                       # CtZone (IPv4)
# registers (pkg/agent/openflow/fields.go)
EP_TO_SELECT = (1 << 16, 0x70000)      # EpToSelectRegMark: reg4[16..18] = 0b001
EP_SELECTED = (2 << 16, 0x70000)       # EpSelectedRegMark: reg4[16..18] = 0b010
EP_UNION_MASK = 0x7ffff                # EpUnionField: reg4[0..18] (EpState + EndpointPort)
REWRITE_MAC = (0x200, 0x200)           # RewriteMACRegMark: reg0[9]
SVC_NO_EP = (0x4000, 0x4000)           # SvcNoEpRegMark: reg0[14]
REMOTE_EP = (0x4000000, 0x4000000)     # RemoteEndpointRegMark: reg4[26]
TO_EXTERNAL = (0x200000, 0x200000)     # ToExternalAddressRegMark: reg4[21]
TO_NODE_PORT = (0x80000, 0x80000)      # ToNodePortAddressRegMark: reg4[19]
VIRTUAL_NODE_PORT_DNAT = "169.254.0.252"  # config.VirtualNodePortDNATIPv4


def _ipv4(ip: str) -> int:
    a = ipaddress.ip_address(ip)
    if a.version != 4:
        raise ValueError("IPv6 Services are not restated (the product rejects them too): %s" % ip)
    return int(a)


def _bucket(i: int, acts: List[str]) -> str:
    return "bucket=bucket_id:%d,weight:100,actions=%s" % (i, ",".join(acts))


class FeatureService:
    """The Service part of openflow.Client: the same install / uninstall calls, flows and groups
    kept in the client's caches and dumped as text."""

    def __init__(self, enable_antrea_policy: bool = True, cookie: int = SERVICE_COOKIE, node_ips=()):
        self.enable_antrea_policy = enable_antrea_policy
        self.cookie = cookie
        self.node_ips = {_ipv4(ip) for ip in node_ips}  # nodeIPChecker.IsNodeIP
        self.cached_flows: Dict[str, List[str]] = {}     # featureService.cachedFlows
        self.groups: Dict[int, str] = {}                 # featureService.groupCache
        # EndpointDNAT is followed by the first egress policy table (pipeline.go stage order)
        self.dnat_next = "AntreaPolicyEgressRule" if enable_antrea_policy else "EgressRule"

    # --- groups (client.go:710-740)
    def install_service_group(self, group_id: int, endpoints: List[dict], with_session_affinity: bool = False):
        head = "group_id=%d,type=select" % group_id
        if not endpoints:
            buckets = [_bucket(0, ["set_field:0x%x/0x%x->reg0" % SVC_NO_EP, "resubmit:EndpointDNAT"])]
        else:
            resubmit = "resubmit:ServiceLB" if with_session_affinity else "resubmit:EndpointDNAT"
            buckets = []
            for i, ep in enumerate(endpoints):
                ip = _ipv4(ep["ip"])
                acts = []
                if not ep.get("is_local") and ep.get("node_name") and ip not in self.node_ips:
                    acts.append("set_field:0x%x/0x%x->reg4" % REMOTE_EP)
                acts.append("set_field:0x%x->reg3" % ip)
                acts.append("set_field:0x%x/0xffff->reg4" % (int(ep["port"]) & 0xffff))
                acts.append(resubmit)
                buckets.append(_bucket(i, acts))
        self.groups[int(group_id)] = ",".join([head] + buckets)

    def uninstall_service_group(self, group_id: int):
        self.groups.pop(int(group_id), None)

    # --- Endpoint flows (client.go:742-788)
    def _endpoint_key(self, ep: dict, protocol: str) -> str:
        return "E%s%s%x" % (ep["ip"], PROTOCOLS[protocol], int(ep["port"]))

    def _endpoint_dnat_flow(self, ip: str, port: int, protocol: str) -> str:
        union = EP_SELECTED[0] + (port & 0xffff)
        return ("cookie=0x%x, table=EndpointDNAT, priority=%d,%s,reg3=0x%x,reg4=0x%x/0x%x "
                "actions=ct(commit,table=%s,zone=%d,nat(dst=%s:%d),exec(set_field:0x10/0x10->ct_mark,"
                "move:NXM_NX_REG0[0..3]->NXM_NX_CT_MARK[0..3]))" % (
                    self.cookie, PRIORITY_NORMAL, PROTOCOLS[protocol], _ipv4(ip), union, EP_UNION_MASK,
                    self.dnat_next, DNAT_CT_ZONE, ip, port))

    def _pod_hairpin_snat_flow(self, ip: str) -> str:
        _ipv4(ip)
        return ("cookie=0x%x, table=SNATMark, priority=%d,ct_state=+new+trk,ip,nw_src=%s,nw_dst=%s "
                "actions=ct(commit,table=SNAT,zone=%d,exec(set_field:0x20/0x20->ct_mark,"
                "set_field:0x40/0x40->ct_mark))" % (self.cookie, PRIORITY_LOW, ip, ip, DNAT_CT_ZONE))

    def install_endpoint_flows(self, protocol: str, endpoints: List[dict]):
        for ep in endpoints:
            flows = [self._endpoint_dnat_flow(ep["ip"], int(ep["port"]), protocol)]
            if ep.get("is_local"):
                flows.append(self._pod_hairpin_snat_flow(ep["ip"]))
            self.cached_flows[self._endpoint_key(ep, protocol)] = flows

    def uninstall_endpoint_flows(self, protocol: str, endpoints: List[dict]):
        for ep in endpoints:
            self.cached_flows.pop(self._endpoint_key(ep, protocol), None)

    # --- Service flows (client.go:790-814)
    # --- NodePortMark (pipeline.go:2282-2314, proxyAll): one flow per non-loopback NodePort address
    # and one for the virtual NodePort DNAT IP
    def set_node_port_addresses(self, ips):
        for k in [k for k in self.cached_flows if k.startswith("NP")]:
            del self.cached_flows[k]
        addrs = [ip for ip in ips if not ipaddress.ip_address(ip).is_loopback]
        if ips:
            addrs.append(VIRTUAL_NODE_PORT_DNAT)
        for ip in addrs:
            self.cached_flows["NP%08x" % _ipv4(ip)] = [
                "cookie=0x%x, table=NodePortMark, priority=%d,ip,nw_dst=%s actions=set_field:0x%x/0x%x->reg4" % (
                    self.cookie, PRIORITY_NORMAL, ip, TO_NODE_PORT[0], TO_NODE_PORT[1])]

    def install_service_flows(self, cfg: dict):
        for k in ("affinity_timeout", "is_dsr", "is_nested"):
            if cfg.get(k):
                raise ValueError("Service shape %s is not restated (the product rejects it too)" % k)
        if cfg.get("is_external") and cfg.get("traffic_policy_local"):  # the short-circuit flow (:2417-2422)
            raise ValueError("external Local Services are not restated (the product rejects them too)")
        proto = cfg["protocol"]
        gid = int(cfg["local_group_id"] if cfg.get("traffic_policy_local") else cfg["cluster_group_id"])
        acts = ["set_field:0x%x/0x%x->reg0" % REWRITE_MAC, "set_field:0x%x/0x%x->reg4" % EP_SELECTED]
        if cfg.get("is_external"):
            acts.append("set_field:0x%x/0x%x->reg4" % TO_EXTERNAL)
        if self.enable_antrea_policy:
            acts.append("set_field:0x%x->reg7" % gid)
        acts.append("group:%d" % gid)
        if cfg.get("is_nodeport"):  # ToNodePortAddressRegMark instead of the Service IP (pipeline.go:2381-2387)
            match = "reg4=0x%x/0x%x" % (EP_TO_SELECT[0] | TO_NODE_PORT[0], EP_TO_SELECT[1] | TO_NODE_PORT[1])
        else:
            match = "reg4=0x%x/0x%x,nw_dst=%s" % (EP_TO_SELECT[0], EP_TO_SELECT[1], cfg["ip"])
        flow = ("cookie=0x%x, table=ServiceLB, priority=%d,%s,%s,tp_dst=%d actions=%s" % (
            self.cookie, PRIORITY_NORMAL, PROTOCOLS[proto], match, int(cfg["port"]), ",".join(acts)))
        _ipv4(cfg["ip"])
        self.cached_flows["S%s%s%x" % (cfg["ip"], PROTOCOLS[proto], int(cfg["port"]))] = [flow]

    def uninstall_service_flows(self, ip: str, port: int, protocol: str):
        self.cached_flows.pop("S%s%s%x" % (ip, PROTOCOLS[protocol], int(port)), None)

    # --- dumps
    def dump_flows(self) -> List[str]:
        return sorted(f for fl in self.cached_flows.values() for f in fl)

    def dump_groups(self) -> List[str]:
        return [self.groups[g] for g in sorted(self.groups)]


def install_services(svc: FeatureService, wl):
    """The AntreaProxy calls for wl's Services, in the order antrea_amd.workload.install_services
    makes them (client.go:710-815: groups, Endpoint flows, Service flows)."""
    if getattr(wl, "node_port_addresses", None):
        svc.set_node_port_addresses(wl.node_port_addresses)
    for gid, eps in wl.groups.items():
        svc.install_service_group(gid, eps)
    for proto, eps in wl.endpoint_flows:
        svc.install_endpoint_flows(proto, eps)
    for cfg in wl.services:
        svc.install_service_flows(cfg)
