"""The reference's e2e policy model restated for verdict pinning (TEST INFRASTRUCTURE ONLY).

The reference pins packet -> verdict behaviour only in its cluster e2e suites
(`test/e2e/antreapolicy_test.go`, `test/e2e/networkpolicy_test.go`): policies are applied to a
fixed Pod universe and every Pod pair is probed (`test/e2e/reachability.go:216-346`,
`k8s_util.go:1068-1119`). This module replays those cases without a cluster:

* `Universe`       -- Namespaces and Pods with labels, IPs and OpenFlow ports, as
                      `k8s_util.go:1147-1196 Bootstrap` creates them (Pod labels pod=<p>, app=<p>;
                      Namespace label ns=<name>; containers c80..c8085 with ports serve-<port>,
                      `k8s_util.go:535-562`). All Pods are local to one Node: a Pod pair's packet is
                      classified by the egress tables (source side) and the ingress tables
                      (destination side) of one pipeline, which is what two Nodes do for it.
* `Controller`     -- the antrea-controller's policy -> internal rule conversion for K8s
                      NetworkPolicy (`pkg/controller/networkpolicy/networkpolicy_controller.go:711-833`,
                      `matchAllPeer :112`, `denyAllRule :1726`), ACNP (`clusternetworkpolicy.go:380-549`,
                      per-Namespace and sameLabels peers) and ANNP (`antreanetworkpolicy.go:98-168`),
                      ClusterGroups / Groups (selectors, ipBlocks, child groups, Service references).
                      Tier priorities: `pkg/controller/networkpolicy/tier.go:47-56`.
* `Reconciler`     -- the agent's podReconciler (`pkg/agent/controller/networkpolicy/pod_reconciler.go`):
                      Reconcile :297-328 (priority registration + ReassignFlowPriorities),
                      computeOFRulesForAdd :521-673, update :715-945 (Add/DeletePolicyRuleAddress),
                      uninstallOFRule / Forget :982-1035 (stale priority release), named ports
                      :1119-1155, address helpers :1157-1258, getOFRuleTable :353-388. It drives any
                      object with the openflow.Client NP surface: the oracle compiler or the product.
* `connectivity`   -- a probe's mark from the two stage verdicts (Connected / Dropped / Rejected;
                      per `k8s_util.go:1089-1101` a pair whose ports disagree is Error).

Rule IDs follow `cache.go:703-729 toRule` + `hashRule`: a rule's identity is its spec (peers by
group name / selector, ipBlocks, Services, action, priorities, appliedTo); group *membership*
changes keep the ID and go through the reconciler's update path, i.e. the churn entry points.
"""
from __future__ import annotations

import ipaddress
import json
from typing import Dict, List, Optional, Tuple

from antrea_amd.caller import PriorityAssigner, ip_blocks_to_of_addresses, of_rule_table

TIERS = {"emergency": 50, "securityops": 100, "networkops": 150, "platform": 200, "application": 250,
         "baseline": 253}
CONTAINER_PORTS = (80, 81, 8080, 8081, 8082, 8083, 8084, 8085)
PROTO_NUM = {"TCP": 6, "UDP": 17, "SCTP": 132, "ICMP": 1}
EPHEMERAL_SPORT = 45678  # inside 32768-60999, the agnhost client's range (antreapolicy_test.go:441-447)

CONNECTED, DROPPED, REJECTED, ERROR = "Con", "Drp", "Rej", "Err"
MARKS = {"Connected": CONNECTED, "Dropped": DROPPED, "Rejected": REJECTED}


# ------------------------------------------------------------------------------------ universe
class Universe:
    def __init__(self, namespaces: Dict[str, Dict[str, str]], pods: Optional[List] = None, family: int = 4):
        self.ns_labels = {}
        for ns, lab in namespaces.items():
            d = dict(lab)
            d["ns"] = ns  # k8s_util.go:1153-1154 convenience label
            d["kubernetes.io/metadata.name"] = ns
            self.ns_labels[ns] = d
        if pods is None:  # antreapolicy_test.go:137-145: pods a, b, c in every Namespace
            pods = [(ns, p, {"pod": p, "app": p}) for p in ("a", "b", "c") for ns in namespaces]
        self.family = family
        self.pods: List[str] = []
        self.labels: Dict[str, Dict[str, str]] = {}
        self.ip: Dict[str, str] = {}
        self.ofport: Dict[str, int] = {}
        for i, (ns, name, lab) in enumerate(sorted(pods, key=lambda t: (t[0], t[1]))):
            key = ns + "/" + name
            self.pods.append(key)
            self.labels[key] = dict(lab)
            self.ip[key] = ("10.10.0.%d" % (i + 1)) if family == 4 else ("fd00:10::%x" % (i + 1))
            self.ofport[key] = 3 + i

    def ns_of(self, pod):
        return pod.split("/", 1)[0]

    def namespaces(self):
        return sorted(self.ns_labels)

    def resolve_ip(self, text: str) -> str:
        """'@x/a' -> that Pod's IP, '@x/a/32' -> its /32 (the e2e code reads podIPs[...] at run time)."""
        if not text.startswith("@"):
            return text
        body = text[1:]
        if body in self.ip:
            return self.ip[body]
        pod, plen = body.rsplit("/", 1)
        return "%s/%s" % (self.ip[pod], plen)


def sel_match(sel: Optional[dict], labels: Dict[str, str]) -> bool:
    """metav1.LabelSelector: {"labels": {...}, "exprs": [[key, op, values]]}; {} selects all."""
    if sel is None:
        return True
    for k, v in (sel.get("labels") or {}).items():
        if labels.get(k) != v:
            return False
    for key, op, values in sel.get("exprs") or []:
        has = key in labels
        if op == "In" and not (has and labels[key] in values):
            return False
        if op == "NotIn" and has and labels[key] in values:
            return False
        if op == "Exists" and not has:
            return False
        if op == "DoesNotExist" and has:
            return False
    return True


# ------------------------------------------------------------------------------------ controller
class Members:
    """An address group's resolution: Pods plus ipBlocks ({"cidr", "except"})."""

    def __init__(self, pods=(), ipblocks=()):
        self.pods = set(pods)
        self.ipblocks = list(ipblocks)

    def union(self, o):
        return Members(self.pods | o.pods, self.ipblocks + o.ipblocks)


MATCH_ALL = [{"cidr": "0.0.0.0/0", "except": []}, {"cidr": "::/0", "except": []}]  # networkpolicy_controller.go:112-117


class Controller:
    """Cluster state (policies, groups, Services, tiers, Pod labels) -> internal rules."""

    def __init__(self, uni: Universe):
        self.u = uni
        self.res: Dict[Tuple[str, str, str], dict] = {}
        self.order: List[Tuple[str, str, str]] = []
        self.tiers = dict(TIERS)

    @staticmethod
    def key(r):
        return (r["kind"], r.get("namespace", ""), r["name"])

    def apply(self, r: dict):
        """CreateOrUpdate (antreapolicy_test.go:4412-4437)."""
        if r["kind"] == "PodLabels":
            self.u.labels[r["name"]] = dict(r["labels"])
            return
        if r["kind"] == "Tier":
            self.tiers[r["name"]] = r["priority"]
            return
        k = self.key(r)
        if k not in self.res:
            self.order.append(k)
        self.res[k] = r

    def delete(self, kind, name, namespace=""):
        k = (kind, namespace, name)
        self.res.pop(k, None)
        if k in self.order:
            self.order.remove(k)

    # --- selection helpers
    def pods_by(self, pod_sel, ns_sel, namespace=None):
        out = set()
        for p in self.u.pods:
            ns = self.u.ns_of(p)
            if namespace is not None and ns != namespace:
                continue
            if ns_sel is not None and not sel_match(ns_sel, self.u.ns_labels[ns]):
                continue
            if not sel_match(pod_sel, self.u.labels[p]):
                continue
            out.add(p)
        return out

    def service_pods(self, ns, name):
        svc = self.res.get(("Service", ns, name))
        if svc is None:
            return set()
        return self.pods_by({"labels": svc["selector"]}, None, namespace=ns)

    def group_members(self, kind, name, namespace="", seen=()):
        """ClusterGroup (cluster scope) / Group (namespaced). A missing group has no members."""
        g = self.res.get((kind, namespace, name))
        if g is None or (kind, name) in seen:
            return Members()
        if g.get("service"):
            return Members(self.service_pods(*g["service"]))
        if g.get("children"):
            m = Members()
            for c in g["children"]:
                m = m.union(self.group_members(kind, c, namespace, seen + ((kind, name),)))
            return m
        if g.get("ipblocks"):
            return Members(ipblocks=[self._ipb(b) for b in g["ipblocks"]])
        if kind == "ClusterGroup":
            return Members(self.pods_by(g.get("pod"), g.get("ns")))
        if g.get("ns") is not None:
            return Members(self.pods_by(g.get("pod"), g.get("ns")))
        return Members(self.pods_by(g.get("pod"), None, namespace=namespace))

    def _ipb(self, b):
        return {"cidr": self.u.resolve_ip(b["cidr"]), "except": [self.u.resolve_ip(e) for e in b.get("except", [])]}

    def _peer(self, p: dict, scope: str, namespace: str) -> Members:
        """One NetworkPolicyPeer. scope: 'cluster' (ACNP), 'ns' (ANNP / K8s NP)."""
        if p.get("ipblock"):
            return Members(ipblocks=[self._ipb(p["ipblock"])])
        if p.get("group"):
            kind = "ClusterGroup" if scope == "cluster" else "Group"
            return self.group_members(kind, p["group"], "" if scope == "cluster" else namespace)
        if p.get("ns") is None and scope == "ns":
            return Members(self.pods_by(p.get("pod"), None, namespace=namespace))
        return Members(self.pods_by(p.get("pod"), p.get("ns")))

    def _applied(self, at: dict, scope: str, namespace: str):
        if at.get("group"):
            kind = "ClusterGroup" if scope == "cluster" else "Group"
            return self.group_members(kind, at["group"], "" if scope == "cluster" else namespace).pods
        if scope == "cluster":
            return self.pods_by(at.get("pod"), at.get("ns"))
        if at.get("ns") is not None:
            return self.pods_by(at.get("pod"), at.get("ns"))
        return self.pods_by(at.get("pod") if at.get("pod") is not None else {}, None, namespace=namespace)

    def _affected_ns(self, at: dict):
        """getAffectedNamespacesForAppliedTo (clusternetworkpolicy.go)."""
        if at.get("ns") is not None:
            return [ns for ns in self.u.namespaces() if sel_match(at["ns"], self.u.ns_labels[ns])]
        return self.u.namespaces()

    # --- internal rules
    def rules(self) -> List[dict]:
        out = []
        for k in self.order:
            r = self.res[k]
            if r["kind"] == "ACNP":
                out += self._acnp(r)
            elif r["kind"] == "ANNP":
                out += self._annp(r)
            elif r["kind"] == "KNP":
                out += self._knp(r)
        return out

    def _base(self, pol, kind, direction, idx, rule, extra):
        ident = {"policy": [kind, pol.get("namespace", ""), pol["name"]], "dir": direction, "idx": idx,
                 "action": rule.get("action", "Allow"), "ports": rule.get("ports"), "name": rule.get("name", ""),
                 "prio": pol.get("priority"), "tier": pol.get("tier")}
        ident.update(extra)
        return ident

    def _mk(self, pol, ptype, direction, idx, rule, peer: Members, applied, ident, max_prio):
        tier = None if ptype == "K8sNetworkPolicy" else self.tiers[pol.get("tier") or "application"]
        ident = dict(ident, tier_priority=tier, ipblocks=peer.ipblocks)
        return {"id": json.dumps(ident, sort_keys=True), "policy_type": ptype, "policy_namespace": pol.get("namespace", ""),
                "policy_name": pol["name"], "policy_uid": "uid-%s-%s" % (pol.get("namespace", ""), pol["name"]),
                "direction": direction, "action": None if ptype == "K8sNetworkPolicy" else rule.get("action", "Allow"),
                "rule_priority": idx, "policy_priority": pol.get("priority"), "tier_priority": tier,
                "max_priority": max_prio, "ports": rule.get("ports"), "name": rule.get("name", ""),
                "peer_pods": set(peer.pods), "peer_ipblocks": peer.ipblocks, "targets": set(applied)}

    def _acnp(self, pol):
        out = []
        max_prio = max([len(pol.get("ingress", [])), len(pol.get("egress", []))]) - 1
        spec_at = pol.get("applied_to") or []
        for direction, rules in (("In", pol.get("ingress", [])), ("Out", pol.get("egress", []))):
            for idx, rule in enumerate(rules):
                peers = rule.get("peers") or []
                cluster = [p for p in peers if not p.get("ns_match")]
                per_ns = [p for p in peers if p.get("ns_match") == "Self"]
                same = [p for p in peers if isinstance(p.get("ns_match"), dict)]
                ats = spec_at if spec_at else (rule.get("applied_to") or [])
                if cluster or not (per_ns or same):
                    applied = set()
                    for at in ats:
                        applied |= self._applied(at, "cluster", "")
                    peer = Members(ipblocks=MATCH_ALL) if not cluster else Members()
                    for p in cluster:
                        peer = peer.union(self._peer(p, "cluster", ""))
                    ident = self._base(pol, "ACNP", direction, idx, rule, {"peers": cluster, "at": ats})
                    out.append(self._mk(pol, "AntreaClusterNetworkPolicy", direction, idx, rule, peer, applied, ident, max_prio))
                if per_ns:
                    for at in ats:
                        for ns in self._affected_ns(at):
                            applied = self.pods_by(at.get("pod"), None, namespace=ns)
                            peer = Members()
                            for p in per_ns:
                                peer = peer.union(Members(self.pods_by(p.get("pod"), None, namespace=ns)))
                            ident = self._base(pol, "ACNP", direction, idx, rule, {"peers": per_ns, "at": at, "ns": ns})
                            out.append(self._mk(pol, "AntreaClusterNetworkPolicy", direction, idx, rule, peer, applied,
                                                ident, max_prio))
                for p in same:
                    labels = p["ns_match"]["same_labels"]
                    groups: Dict[tuple, List[str]] = {}
                    for at in ats:
                        for ns in self._affected_ns(at):
                            nl = self.u.ns_labels[ns]
                            if all(l in nl for l in labels):
                                groups.setdefault(tuple(nl[l] for l in labels), []).append(ns)
                    for vals, nss in sorted(groups.items()):
                        applied, peer = set(), Members()
                        for ns in nss:
                            for at in ats:
                                applied |= self.pods_by(at.get("pod"), None, namespace=ns)
                            peer = peer.union(Members(self.pods_by(p.get("pod"), None, namespace=ns)))
                        ident = self._base(pol, "ACNP", direction, idx, rule, {"peers": [p], "at": ats, "vals": list(vals)})
                        out.append(self._mk(pol, "AntreaClusterNetworkPolicy", direction, idx, rule, peer, applied, ident,
                                            max_prio))
        return out

    def _annp(self, pol):
        out = []
        ns = pol["namespace"]
        max_prio = max([len(pol.get("ingress", [])), len(pol.get("egress", []))]) - 1
        for direction, rules in (("In", pol.get("ingress", [])), ("Out", pol.get("egress", []))):
            for idx, rule in enumerate(rules):
                ats = rule.get("applied_to") or pol.get("applied_to") or []
                applied = set()
                for at in ats:
                    applied |= self._applied(at, "ns", ns)
                peers = rule.get("peers") or []
                peer = Members(ipblocks=MATCH_ALL) if not peers else Members()
                for p in peers:
                    peer = peer.union(self._peer(p, "ns", ns))
                ident = self._base(pol, "ANNP", direction, idx, rule, {"peers": peers, "at": ats})
                out.append(self._mk(pol, "AntreaNetworkPolicy", direction, idx, rule, peer, applied, ident, max_prio))
        return out

    def _knp(self, pol):
        out = []
        ns = pol["namespace"]
        applied = self.pods_by(pol.get("pod_selector") or {}, None, namespace=ns)
        types = pol.get("types") or []
        for direction, rules, t in (("In", pol.get("ingress"), "Ingress"), ("Out", pol.get("egress"), "Egress")):
            if rules:
                for idx, rule in enumerate(rules):
                    peers = rule.get("peers") or []
                    peer = Members(ipblocks=MATCH_ALL) if not peers else Members()
                    for p in peers:
                        peer = peer.union(self._peer(p, "ns", ns))
                    ident = self._base(pol, "KNP", direction, idx, rule, {"peers": peers, "sel": pol.get("pod_selector")})
                    out.append(self._mk(pol, "K8sNetworkPolicy", direction, -1, rule, peer, applied, ident, -1))
            elif t in types:  # denyAllRule (networkpolicy_controller.go:768-777, 1726-1731)
                ident = self._base(pol, "KNP", direction, "denyall", {}, {"sel": pol.get("pod_selector")})
                out.append(self._mk(pol, "K8sNetworkPolicy", direction, -1, {"ports": None}, Members(), applied, ident, -1))
        return out


# ------------------------------------------------------------------------------------ reconciler
def _services(ports, member_ports=None):
    """v1beta2.Service list (None = all ports). A named port resolves against the member's
    container ports (resolveService, pod_reconciler.go:1285-1310): containers listen on TCP."""
    if ports is None:
        return None
    out = []
    for p in ports:
        s = {"protocol": p.get("protocol", "TCP")}
        if p.get("port_name") is not None:
            if member_ports is None or s["protocol"] != "TCP":
                s["port_name"] = p["port_name"]
            else:
                num = int(p["port_name"].split("-")[1])
                if num in member_ports:
                    s["port"] = num
                else:
                    s["port_name"] = p["port_name"]
        for f in ("port", "end_port", "src_port", "src_end_port", "icmp_type", "icmp_code"):
            if p.get(f) is not None:
                s[f] = p[f]
        out.append(s)
    return out


def _svc_key(svcs):
    """normalizeServices (pod_reconciler.go:87-99)."""
    if not svcs:
        return ""
    return ",".join(str(s.get("port", 0)) for s in svcs)


def _filter_unresolvable(svcs):
    """filterUnresolvablePort (pod_reconciler.go:1260-1281)."""
    if not svcs:
        return None
    return [s for s in svcs if "port_name" not in s]


class Reconciler:
    """podReconciler over an openflow.Client NP surface (oracle compiler or product)."""

    TABLES = ("AntreaPolicyIngressRule", "AntreaPolicyEgressRule", "IngressDefaultRule", "EgressDefaultRule")

    def __init__(self, client, uni: Universe):
        self.c = client
        self.u = uni
        self.assigners = {t: PriorityAssigner(is_baseline=t.endswith("DefaultRule")) for t in self.TABLES}
        self.realized: Dict[str, dict] = {}
        self.next_id = 1
        self.conj_policy: Dict[int, Tuple[str, str]] = {}
        self.conj_tier: Dict[int, int] = {}
        self.log: List[tuple] = []  # (openflow.Client call, rule id / flow id) -- what the step drove

    def _table(self, r):
        return of_rule_table(r["direction"], r["policy_type"] != "K8sNetworkPolicy", r["tier_priority"])

    def _ips(self, pods):
        return sorted(self.u.ip[p] for p in pods)

    def _of_priority(self, r, table):
        """getOFPriority (pod_reconciler.go:392-430)."""
        if r["policy_type"] == "K8sNetworkPolicy":
            return None
        pa = self.assigners[table]
        p = (r["tier_priority"], r["policy_priority"], r["rule_priority"])
        of, ok = pa.get_of_priority(p)
        if not ok:
            allp = [(r["tier_priority"], r["policy_priority"], i) for i in range(r["max_priority"] + 1)]
            updates, _ = pa.register_priorities(allp)
            if updates:
                self.c.reassign_flow_priorities(updates, table)
                self.log.append(("ReassignFlowPriorities", table, dict(updates)))
            of, _ = pa.get_of_priority(p)
        return of

    def _rule_dict(self, r, table, prio, direction, frm, to, svcs):
        d = {"direction": direction, "table": table, "from": frm, "to": to, "flow_id": None,
             "policy_type": r["policy_type"], "policy_namespace": r["policy_namespace"],
             "policy_name": r["policy_name"], "policy_uid": r["policy_uid"], "name": r["name"]}
        if svcs is not None:
            d["service"] = svcs
        if r["action"] is not None:
            d["action"] = r["action"]
        if prio is not None:
            d["priority"] = prio
        if r["tier_priority"] is not None:
            d["tier_priority"] = r["tier_priority"]
        return d

    def _install(self, r, d):
        """installOFRule (pod_reconciler.go:947-954) with idAllocator.allocateForRule."""
        d["flow_id"] = self.next_id
        self.conj_policy[self.next_id] = (r["policy_name"], r["policy_type"])
        self.conj_tier[self.next_id] = int(r["tier_priority"] or 0)
        self.next_id += 1
        self.c.install_policy_rule_flows(d)
        self.log.append(("InstallPolicyRuleFlows", d["flow_id"]))
        return d["flow_id"]

    def _by_services(self, ports, members):
        """groupMembersByServices (pod_reconciler.go:1119-1155)."""
        named = any(p.get("port_name") for p in (ports or []))
        if not named:
            svcs = _services(ports)
            return {_svc_key(svcs): (set(members), svcs)}
        out = {}
        for m in sorted(members):
            svcs = _services(ports, CONTAINER_PORTS)
            k = _svc_key(svcs)
            out.setdefault(k, (set(), svcs))[0].add(m)
        return out

    def _compute(self, r, table, prio):
        """computeOFRulesForAdd (pod_reconciler.go:521-673) -> {svcKey: (PolicyRule dict, state)}."""
        out = {}
        fam4 = self.u.family == 4
        ipb = ip_blocks_to_of_addresses(r["peer_ipblocks"], ipv4=fam4, ipv6=not fam4)
        if r["direction"] == "In":
            frm = self._ips(r["peer_pods"]) + ipb
            for k, (members, svcs) in self._by_services(r["ports"], r["targets"]).items():
                to = [{"ofport": self.u.ofport[p]} for p in sorted(members)]
                out[k] = (self._rule_dict(r, table, prio, "In", frm, to, _filter_unresolvable(svcs)),
                          {"from": set(r["peer_pods"]), "to": set(members)})
        else:
            frm = self._ips(r["targets"])
            for k, (members, svcs) in self._by_services(r["ports"], r["peer_pods"]).items():
                out[k] = (self._rule_dict(r, table, prio, "Out", frm, self._ips(members), _filter_unresolvable(svcs)),
                          {"from": set(r["targets"]), "to": set(members)})
            if r["policy_type"] == "K8sNetworkPolicy" or r["peer_ipblocks"]:
                k = _svc_key(_services(r["ports"]))
                if k not in out:
                    out[k] = (self._rule_dict(r, table, prio, "Out", frm, [], _filter_unresolvable(_services(r["ports"]))),
                              {"from": set(r["targets"]), "to": set()})
                out[k][0]["to"] = out[k][0]["to"] + ipb
        return out

    def sync(self, rules: List[dict]):
        """One step: Forget rules that disappeared, Reconcile (add / update) the rest."""
        want = {r["id"]: r for r in rules}
        for rid in [k for k in self.realized if k not in want]:
            self._forget(rid)
        for r in rules:
            self._reconcile(r)

    def _reconcile(self, r):
        table = self._table(r)
        prio = self._of_priority(r, table)
        last = self.realized.get(r["id"])
        if last is None:
            ofr = self._compute(r, table, prio)
            for k, (d, _) in ofr.items():
                self._install(r, d)
            self.realized[r["id"]] = {"rule": r, "table": table, "ids": {k: d["flow_id"] for k, (d, _) in ofr.items()},
                                      "state": {k: s for k, (_, s) in ofr.items()}}
            return
        self._update(last, r, table, prio)

    def _update(self, last, r, table, prio):
        """update (pod_reconciler.go:715-945) for Pod members: address diffs per svcKey."""
        fresh = self._compute(r, table, prio)
        stale = dict(last["ids"])
        for k, (d, st) in fresh.items():
            if k not in last["ids"]:
                last["ids"][k] = self._install(r, d)
                last["state"][k] = st
                continue
            fid = last["ids"][k]
            old = last["state"][k]
            if r["direction"] == "In":
                add_f, del_f = st["from"] - old["from"], old["from"] - st["from"]
                add_t = [{"ofport": self.u.ofport[p]} for p in sorted(st["to"] - old["to"])]
                del_t = [{"ofport": self.u.ofport[p]} for p in sorted(old["to"] - st["to"])]
            else:
                add_f, del_f = st["from"] - old["from"], old["from"] - st["from"]
                add_t, del_t = self._ips(st["to"] - old["to"]), self._ips(old["to"] - st["to"])
            calls = (("src", self._ips(add_f), True), ("dst", add_t, True), ("src", self._ips(del_f), False),
                     ("dst", del_t, False))
            for typ, addrs, add in calls:  # updateOFRule order (pod_reconciler.go:956-980)
                if not addrs:
                    continue
                if add:
                    self.c.add_policy_rule_address(fid, typ, addrs, prio)
                    self.log.append(("AddPolicyRuleAddress", fid, typ, len(addrs)))
                else:
                    self.c.delete_policy_rule_address(fid, typ, addrs, prio)
                    self.log.append(("DeletePolicyRuleAddress", fid, typ, len(addrs)))
            last["state"][k] = st
            stale.pop(k)
        for k, fid in stale.items():
            self._uninstall(fid, table)
            del last["ids"][k]
            del last["state"][k]
        last["rule"] = r

    def _uninstall(self, fid, table):
        """uninstallOFRule (pod_reconciler.go:982-1003): release stale OF priorities."""
        stale = self.c.uninstall_policy_rule_flows(fid)
        self.log.append(("UninstallPolicyRuleFlows", fid))
        if stale and table in self.assigners:
            for p in stale:
                self.assigners[table].release(int(p))

    def _forget(self, rid):
        last = self.realized.pop(rid)
        for fid in last["ids"].values():
            self._uninstall(fid, last["table"])


# ------------------------------------------------------------------------------------ probes
def expected_matrix(uni: Universe, ops: List[list]) -> Dict[Tuple[str, str], str]:
    """Replay reachability.go's Expect* calls (reachability.go:216-346) into a full matrix."""
    m: Dict[Tuple[str, str], str] = {}
    by_ns: Dict[str, List[str]] = {}
    for p in uni.pods:
        by_ns.setdefault(uni.ns_of(p), []).append(p)
    for op in ops:
        kind, args = op[0], op[1:]
        mark = MARKS[args[-1]]
        if kind == "new":
            m = {(a, b): mark for a in uni.pods for b in uni.pods}
        elif kind == "expect":
            m[(args[0], args[1])] = mark
        elif kind == "self":
            for p in uni.pods:
                m[(p, p)] = mark
        elif kind == "all_ingress":
            for a in uni.pods:
                m[(a, args[0])] = mark
        elif kind == "all_egress":
            for b in uni.pods:
                m[(args[0], b)] = mark
        elif kind == "all_self_ns":
            for pods in by_ns.values():
                for a in pods:
                    for b in pods:
                        m[(a, b)] = mark
        elif kind == "self_ns":
            for a in by_ns[args[0]]:
                for b in by_ns[args[0]]:
                    m[(a, b)] = mark
        elif kind == "ingress_from_ns":
            for a in by_ns[args[1]]:
                m[(a, args[0])] = mark
        elif kind == "egress_to_ns":
            for b in by_ns[args[1]]:
                m[(args[0], b)] = mark
        elif kind == "ns_ingress_from_ns":
            for d in by_ns[args[0]]:
                for a in by_ns[args[1]]:
                    m[(a, d)] = mark
        elif kind == "probe":  # a single client -> server probe (networkpolicy_test.go)
            m[(args[0], args[1])] = mark
        elif kind == "ns_egress_to_ns":
            for s in by_ns[args[0]]:
                for b in by_ns[args[1]]:
                    m[(s, b)] = mark
        else:
            raise ValueError(kind)
    return m


def probe_packets(uni: Universe, pairs, ports, protocol):
    """Packet per (pair, port): the first packet of the probe's connection (ct_state +new+trk),
    as the source Node's egress tables and the destination Node's ingress tables see it."""
    pkts = []
    for (a, b) in pairs:
        for port in ports:
            pkts.append({"src": a, "dst": b, "port": port, "proto": PROTO_NUM[protocol]})
    return pkts


ACT_NONE, ACT_NO_MATCH, ACT_ALLOW, ACT_DROP, ACT_REJECT, ACT_ISOLATION_DROP, ACT_BYPASS = range(7)


def connectivity(e_act: int, i_act: int) -> str:
    """A probe's mark from the two stages: a Drop / isolation drop in either stage drops the
    connection, a Reject rejects it (REJECT packet-in, `pipeline.go:1812-1859`); else it connects."""
    for a in (e_act, i_act):
        if a == ACT_REJECT:
            return REJECTED
        if a in (ACT_DROP, ACT_ISOLATION_DROP):
            return DROPPED
    return CONNECTED


def deciding(e, i):
    """(stage verdict tuple) of the rule that decided a probe: a dropping / rejecting stage, else the
    ingress allow, else the egress allow (NetworkPolicyEvaluation's answer for these cases)."""
    if e[0] in (ACT_DROP, ACT_REJECT, ACT_ISOLATION_DROP):
        return e
    if i[0] in (ACT_DROP, ACT_REJECT, ACT_ISOLATION_DROP):
        return i
    if i[0] == ACT_ALLOW:
        return i
    if e[0] == ACT_ALLOW:
        return e
    return None


EVAL_ACTION = {"Allow": ACT_ALLOW, "Drop": ACT_DROP, "Reject": ACT_REJECT, "Isolate": ACT_ISOLATION_DROP}
