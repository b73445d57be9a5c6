"""Hand translation of the reference's e2e reachability cases (TEST INFRASTRUCTURE ONLY).

Each case restates one `test/e2e/antreapolicy_test.go` (or `networkpolicy_test.go`) test function:
the policies / groups / Services its steps apply, in a declarative form the model of
`tests/e2e_model.py` understands, and the expectations of its steps exactly as the Go code writes
them (`reachability.go` calls: NewReachability / Expect / ExpectSelf / ExpectAllIngress / ...,
and `NPEvaluation.Expect / ExpectNone`). `src` names the Go variable and the line range holding
a step's reachability calls; `make_e2e_reachability.py` parses those lines out of the reference
and refuses to write the fixture unless they equal the transcription here (the policies are
transcribed by hand; the builder argument positions are noted where they matter).

Notation: selectors are {"labels": {...}, "exprs": [[key, op, values]]}; a pod is "ns/name";
"@ns/name" in an ipBlock is that Pod's IP (the Go code reads it from podIPs at run time).
"""

GO = "test/e2e/antreapolicy_test.go"
GO_NP = "test/e2e/networkpolicy_test.go"


def S(**labels):
    return {"labels": labels}


def NS(n):
    return {"labels": {"ns": n}}


def POD(p):
    return {"labels": {"pod": p}}


ALL = {"labels": {}}  # map[string]string{} selector: everything


def port(p=None, proto="TCP", end=None, name=None, sport=None, send=None):
    d = {"protocol": proto}
    if p is not None:
        d["port"] = p
    if end is not None:
        d["end_port"] = end
    if name is not None:
        d["port_name"] = name
    if sport is not None:
        d["src_port"] = sport
    if send is not None:
        d["src_end_port"] = send
    return d


def rule(action="Allow", ports=None, peers=(), at=None, name=""):
    r = {"action": action, "ports": ports, "peers": list(peers), "name": name}
    if at:
        r["applied_to"] = list(at)
    return r


def peer(pod=None, ns=None, ipblock=None, group=None, ns_match=None):
    d = {}
    if pod is not None:
        d["pod"] = pod
    if ns is not None:
        d["ns"] = ns
    if ipblock is not None:
        d["ipblock"] = ipblock
    if group is not None:
        d["group"] = group
    if ns_match is not None:
        d["ns_match"] = ns_match
    return d


def at(pod=None, ns=None, group=None):
    d = {}
    if pod is not None:
        d["pod"] = pod
    if ns is not None:
        d["ns"] = ns
    if group is not None:
        d["group"] = group
    return d


def acnp(name, prio, applied=None, ingress=(), egress=(), tier=None):
    return {"kind": "ACNP", "name": name, "priority": prio, "tier": tier, "applied_to": list(applied or []),
            "ingress": list(ingress), "egress": list(egress)}


def annp(ns, name, prio, applied=None, ingress=(), egress=(), tier=None):
    return {"kind": "ANNP", "namespace": ns, "name": name, "priority": prio, "tier": tier,
            "applied_to": list(applied or []), "ingress": list(ingress), "egress": list(egress)}


def knp(ns, name, pod_selector=None, types=(), ingress=None, egress=None):
    return {"kind": "KNP", "namespace": ns, "name": name, "pod_selector": pod_selector or {}, "types": list(types),
            "ingress": ingress, "egress": egress}


def kpeer(pod=None, ns=None, cidr=None, except_=()):
    d = {}
    if pod is not None:
        d["pod"] = pod
    if ns is not None:
        d["ns"] = ns
    if cidr is not None:
        d["ipblock"] = {"cidr": cidr, "except": list(except_)}
    return d


def cg(name, pod=None, ns=None, ipblocks=None, children=None, service=None):
    return {"kind": "ClusterGroup", "name": name, "pod": pod, "ns": ns, "ipblocks": ipblocks, "children": children,
            "service": service}


def grp(ns, name, pod=None, nsel=None, ipblocks=None, children=None, service=None):
    return {"kind": "Group", "namespace": ns, "name": name, "pod": pod, "ns": nsel, "ipblocks": ipblocks,
            "children": children, "service": service}


def svc(ns, name, selector):
    return {"kind": "Service", "namespace": ns, "name": name, "selector": selector}


def step(name, apply, reach, src, ports=(80,), protocol="TCP", evaluation=(), delete=(), eval_src=None):
    d = {"name": name, "apply": list(apply), "delete": list(delete), "reach": [list(o) for o in reach], "src": list(src),
         "ports": list(ports), "protocol": protocol, "eval": [list(e) for e in evaluation]}
    if eval_src:
        d["eval_src"] = list(eval_src)
    return d


def case(name, go_func, steps, base=(), universe="xyz", go_file=GO):
    return {"name": name, "go_func": go_func, "go_file": go_file, "universe": universe, "base": list(base),
            "steps": list(steps)}


# antreapolicy_test.go:161-181 applyDefaultDenyToAllNamespaces (TestGroupDefaultDENY, :4603-4610)
DEFAULT_DENY = [knp(n, "default-deny-namespace", {}, ["Ingress"]) for n in ("x", "y", "z")]
TCP80 = [port(80)]

CASES = []

# ---------------------------------------------------------------------------------------- :412
CASES.append(case("ACNP Allow X/B to A", "testACNPAllowXBtoA", base=DEFAULT_DENY, steps=[
    step("Port 80", [acnp("acnp-allow-xb-to-a", 1.0, [at(pod=POD("a"))],
                          ingress=[rule("Allow", TCP80, [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Dropped"), ("expect", "x/b", "x/a", "Connected"), ("expect", "x/b", "y/a", "Connected"),
          ("expect", "x/b", "z/a", "Connected"), ("self", "Connected")], ("reachability", 420, 424))]))

# ---------------------------------------------------------------------------------------- :508 (named port)
CASES.append(case("ACNP Allow X/B to Y/A", "testACNPAllowXBtoYA", base=DEFAULT_DENY, steps=[
    step("NamedPort 81", [acnp("acnp-allow-xb-to-ya", 2.0, [at(pod=POD("a"), ns=NS("y"))],
                               ingress=[rule("Allow", [port(name="serve-81")], [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Dropped"), ("expect", "x/b", "y/a", "Connected"), ("self", "Connected")],
         ("reachability", 517, 519), ports=(81,))]))

# ---------------------------------------------------------------------------------------- :539 (+ evaluation)
_p2 = acnp("acnp-priority2", 2, [at(ns=NS("x"))], ingress=[rule("Allow", TCP80, [peer(ns=NS("z"))])])
_p1 = acnp("acnp-priority1", 1, [at(pod=POD("a"), ns=NS("x"))], ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])])
CASES.append(case("ACNP PriorityOverride Default Deny", "testACNPPriorityOverrideDefaultDeny", base=DEFAULT_DENY, steps=[
    step("Both ACNP", [_p2, _p1],
         [("new", "Dropped")] + [("expect", "z/%s" % s, "x/%s" % d, "Connected") for s in "abc" for d in "bc"] +
         [("self", "Connected")], ("reachabilityBothACNP", 555, 562),
         evaluation=[("y/a", "x/a", "default-deny-namespace", "Isolate"), ("z/b", "x/a", "acnp-priority1", "Drop"),
                     ("z/b", "x/b", "acnp-priority2", "Allow")], eval_src=("evaluationBothACNPs", 564, 567))]))

# ---------------------------------------------------------------------------------------- :586
for _proto in ("TCP", "UDP", "SCTP"):
    CASES.append(case("ACNP Allow No Default Isolation " + _proto, "testACNPAllowNoDefaultIsolation", steps=[
        step("Port 81", [acnp("acnp-allow-x-ingress-y-egress-z", 1.1, [at(ns=NS("x"))],
                              ingress=[rule("Allow", [port(81, _proto)], [peer(ns=NS("y"))])],
                              egress=[rule("Allow", [port(81, _proto)], [peer(ns=NS("z"))])])],
             [("new", "Connected")], ("reachability", 604, 604), ports=(81,), protocol=_proto)]))

# ---------------------------------------------------------------------------------------- :621
for _proto in ("TCP", "UDP", "SCTP"):
    CASES.append(case("ACNP Drop Egress From All Pod:a to NS:z " + _proto, "testACNPDropEgress", steps=[
        step("Port 80", [acnp("acnp-deny-a-to-z-egress", 1.0, [at(pod=POD("a"))],
                              egress=[rule("Drop", [port(80, _proto)], [peer(ns=NS("z"))])])],
             [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
              ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 637, 641),
             protocol=_proto)]))

# ---------------------------------------------------------------------------------------- :660 (empty From)
CASES.append(case("ACNP Drop all Ingress to Namespace x", "testACNPDropIngressInSelectedNamespace", steps=[
    step("Port 80", [acnp("acnp-deny-ingress-to-x", 1.0, [at(ns=NS("x"))],
                          ingress=[rule("Drop", TCP80, [], name="drop-all-ingress")])],
         [("new", "Connected"), ("all_ingress", "x/a", "Dropped"), ("all_ingress", "x/b", "Dropped"),
          ("all_ingress", "x/c", "Dropped"), ("self", "Connected")], ("reachability", 668, 672))]))

# ---------------------------------------------------------------------------------------- :688 (ipBlock except)
_ipb_except = acnp("acnp-drop-all-egress-from-ya-except-xa-xb-ip", 1.0, [at(pod=POD("a"), ns=NS("y"))],
                   egress=[rule("Drop", TCP80, [peer(ipblock={"cidr": "0.0.0.0/0", "except": ["@x/a/32", "@x/b/32"]})],
                                name="egress-drop-0")])
CASES.append(case("ACNP Drop rule with a ipBlock that has except clause", "testACNPDropIPBlockWithExcept", steps=[
    step("Port 80", [_ipb_except],
         [("new", "Connected"), ("all_egress", "y/a", "Dropped"), ("expect", "y/a", "x/a", "Connected"),
          ("expect", "y/a", "x/b", "Connected"), ("expect", "y/a", "y/a", "Connected")], ("reachability", 700, 704))]))
CASES.append(case("ACNP Drop rule with a ipBlock that has except clause and underlying Drop rules",
                  "testACNPDropIPBlockWithExcept", steps=[
    step("Port 80", [_ipb_except, acnp("acnp-drop-egress-from-ya-to-xa", 2.0, [at(pod=POD("a"), ns=NS("y"))],
                                       egress=[rule("Drop", TCP80, [peer(pod=POD("a"), ns=NS("x"))], name="egress-drop-xa")])],
         [("new", "Connected"), ("all_egress", "y/a", "Dropped"), ("expect", "y/a", "x/b", "Connected"),
          ("expect", "y/a", "y/a", "Connected")], ("reachability2", 721, 724))]))

# ---------------------------------------------------------------------------------------- :742
_noeff = acnp("acnp-deny-a-to-z-ingress", 1.0, [at(pod=POD("a"))], ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])])
CASES.append(case("ACNP Drop Ingress From All Pod:a to NS:z TCP Not UDP", "testACNPNoEffectOnOtherProtocols", steps=[
    step("Port 80", [_noeff],
         [("new", "Connected")] + [("expect", "z/%s" % s, "%s/a" % d, "Dropped") for d, srcs in (("x", "abc"), ("y", "abc"))
                                   for s in srcs] +
         [("expect", "z/b", "z/a", "Dropped"), ("expect", "z/c", "z/a", "Dropped")], ("reachability1", 750, 758)),
    step("Port 80 UDP", [_noeff], [("new", "Connected")], ("reachability2", 760, 760), protocol="UDP")]))

# ---------------------------------------------------------------------------------------- :785 / :820 (CG, named port)
CASES.append(case("ACNP Deny ClusterGroup Y/A from X/B", "testACNPAppliedToDenyXBtoCGWithYA", steps=[
    step("NamedPort 81", [acnp("acnp-deny-cg-with-ya-from-xb", 2.0, [at(group="cg-pods-ya")],
                               ingress=[rule("Drop", [port(name="serve-81")], [peer(pod=POD("b"), ns=NS("x"))])]),
                          cg("cg-pods-ya", pod=POD("a"), ns=NS("y"))],
         [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped"), ("self", "Connected")],
         ("reachability", 799, 801), ports=(81,))]))
CASES.append(case("ACNP Deny ClusterGroup X/B to Y/A", "testACNPIngressRuleDenyCGWithXBtoYA", steps=[
    step("NamedPort 81", [cg("cg-pods-xb", pod=POD("b"), ns=NS("x")),
                          acnp("acnp-deny-cg-with-xb-to-ya", 2.0, [at(pod=POD("a"), ns=NS("y"))],
                               ingress=[rule("Drop", [port(name="serve-81")], [peer(group="cg-pods-xb")])])],
         [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped"), ("self", "Connected")],
         ("reachability", 834, 836), ports=(81,))]))

# ---------------------------------------------------------------------------------------- :854 / :886
CASES.append(case("ACNP Drop Egress From ClusterGroup with All Pod:a to NS:z", "testACNPAppliedToRuleCGWithPodsAToNsZ", steps=[
    step("Port 80", [acnp("acnp-deny-cg-with-a-to-z", 1.0, None,
                          egress=[rule("Drop", TCP80, [peer(ns=NS("z"))], at=[at(group="cg-pods-a")])]),
                     cg("cg-pods-a", pod=POD("a"))],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
          ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 864, 868))]))
CASES.append(case("ACNP Drop Egress From All Pod:a to ClusterGroup with NS:z", "testACNPEgressRulePodsAToCGWithNsZ", steps=[
    step("Port 80", [acnp("acnp-deny-a-to-cg-with-z-egress", 1.0, [at(pod=POD("a"))],
                          egress=[rule("Drop", TCP80, [peer(group="cg-ns-z")])]),
                     cg("cg-ns-z", ns=NS("z"))],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
          ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 897, 901))]))

# ---------------------------------------------------------------------------------------- :918 / :965 (CG updates)
CASES.append(case("ACNP Drop Egress From CG Pod:a to NS:z updated to ClusterGroup with Pod:c",
                  "testACNPClusterGroupUpdateAppliedTo", steps=[
    step("CG Pods A", [cg("cg-pods-a-then-c", pod=POD("a")),
                       acnp("acnp-deny-cg-with-a-to-z-egress", 1.0, [at(group="cg-pods-a-then-c")],
                            egress=[rule("Drop", TCP80, [peer(ns=NS("z"))])])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
          ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 932, 936)),
    step("CG Pods C - update", [cg("cg-pods-a-then-c", pod=POD("c"))],
         [("new", "Connected"), ("egress_to_ns", "x/c", "z", "Dropped"), ("egress_to_ns", "y/c", "z", "Dropped"),
          ("expect", "z/c", "z/a", "Dropped"), ("expect", "z/c", "z/b", "Dropped")], ("updatedReachability", 938, 942))]))
CASES.append(case("ACNP Drop Egress From All Pod:a to ClusterGroup with NS:z updated to ClusterGroup with NS:y",
                  "testACNPClusterGroupUpdate", steps=[
    step("Port 80", [cg("cg-ns-z-then-y", ns=NS("z")),
                     acnp("acnp-deny-a-to-cg-with-z-egress", 1.0, [at(pod=POD("a"))],
                          egress=[rule("Drop", TCP80, [peer(group="cg-ns-z-then-y")])])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
          ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 979, 983)),
    step("Port 80 - update", [cg("cg-ns-z-then-y", ns=NS("y"))],
         [("new", "Connected"), ("egress_to_ns", "x/a", "y", "Dropped"), ("egress_to_ns", "z/a", "y", "Dropped"),
          ("expect", "y/a", "y/b", "Dropped"), ("expect", "y/a", "y/c", "Dropped")], ("updatedReachability", 985, 989))]))

# ---------------------------------------------------------------------------------------- :1139 (CG ipBlocks)
CASES.append(case("ACNP Drop Ingress From x to Pod y/a to ClusterGroup with ipBlocks", "testACNPClusterGroupRefRuleIPBlocks",
                  steps=[
    step("Port 80", [acnp("acnp-deny-x-ips-ingress-for-ya", 1.0, [at(pod=POD("a"), ns=NS("y"))],
                          ingress=[rule("Drop", TCP80, [peer(group="cg-ipblocks-pod-in-ns-x")]),
                                   rule("Drop", TCP80, [peer(group="cg-ipblock-pod-za")])]),
                     cg("cg-ipblocks-pod-in-ns-x", ipblocks=[{"cidr": "@x/%s/32" % p} for p in "abc"]),
                     cg("cg-ipblock-pod-za", ipblocks=[{"cidr": "@z/a/32"}])],
         [("new", "Connected"), ("expect", "x/a", "y/a", "Dropped"), ("expect", "x/b", "y/a", "Dropped"),
          ("expect", "x/c", "y/a", "Dropped"), ("expect", "z/a", "y/a", "Dropped")], ("reachability", 1174, 1178))]))

# ---------------------------------------------------------------------------------------- ANNP + Group :1195-1437
CASES.append(case("ANNP Drop Egress From All Pod:x/a to Group with Pod:x/c", "testANNPEgressRulePodsAToGrpWithPodsC", steps=[
    step("Port 80", [annp("x", "annp-deny-xa-to-grp-xc-egress", 1.0, [at(pod=POD("a"))],
                          egress=[rule("Drop", TCP80, [peer(group="grp-xc")])]),
                     grp("x", "grp-xc", pod=POD("c"))],
         [("new", "Connected"), ("expect", "x/a", "x/c", "Dropped")], ("reachability", 1206, 1207))]))
CASES.append(case("ANNP Deny Group X/B to X/A", "testANNPIngressRuleDenyGrpWithXCtoXA", steps=[
    step("NamedPort 81", [grp("x", "grp-pods-xb", pod=POD("b")),
                          annp("x", "annp-deny-grp-with-xb-to-xa", 2.0, [at(pod=POD("a"))],
                               ingress=[rule("Drop", [port(name="serve-81")], [peer(group="grp-pods-xb")])])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("self", "Connected")],
         ("reachability", 1237, 1239), ports=(81,))]))
CASES.append(case("ANNP Drop Egress From All Pod:x/a to Group with Pod:x/c updated to Group with Pod:x/b",
                  "testANNPGroupUpdate", steps=[
    step("Port 80", [grp("x", "grp-pod-xc-then-pod-xb", pod=POD("c")),
                     annp("x", "annp-deny-xa-to-grp-with-xc-egress", 1.0, [at(pod=POD("a"))],
                          egress=[rule("Drop", TCP80, [peer(group="grp-pod-xc-then-pod-xb")])])],
         [("new", "Connected"), ("expect", "x/a", "x/c", "Dropped")], ("reachability", 1270, 1271)),
    step("Port 80 - update", [grp("x", "grp-pod-xc-then-pod-xb", pod=POD("b"))],
         [("new", "Connected"), ("expect", "x/a", "x/b", "Dropped")], ("updatedReachability", 1273, 1274))]))
CASES.append(case("ANNP Deny Group X/A from X/B", "testANNPAppliedToDenyXBtoGrpWithXA", steps=[
    step("NamedPort 81", [annp("x", "annp-deny-grp-with-xa-from-xb", 2.0, [at(group="grp-pods-ya")],
                               ingress=[rule("Drop", [port(name="serve-81")], [peer(pod=POD("b"))])]),
                          grp("x", "grp-pods-ya", pod=POD("a"))],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("self", "Connected")],
         ("reachability", 1310, 1312), ports=(81,))]))
CASES.append(case("ANNP Drop Egress From Group with All Pod:a to Pod:c", "testANNPAppliedToRuleGrpWithPodsAToPodsC", steps=[
    step("Port 80", [annp("x", "annp-deny-grp-with-a-to-c", 1.0, None,
                          egress=[rule("Drop", TCP80, [peer(pod=POD("c"))], at=[at(group="grp-pods-a")])]),
                     grp("x", "grp-pods-a", pod=POD("a"))],
         [("new", "Connected"), ("expect", "x/a", "x/c", "Dropped")], ("reachability", 1341, 1342))]))
CASES.append(case("ANNP Drop Egress From Pod:x/c to Group Pod:x/a updated to Group with Pod:x/b",
                  "testANNPGroupUpdateAppliedTo", steps=[
    step("GRP Pods X/C", [grp("x", "grp-pods-xa-then-xb", pod=POD("a")),
                          annp("x", "annp-deny-grp-xc-to-xa-egress", 1.0, [at(group="grp-pods-xa-then-xb")],
                               egress=[rule("Drop", TCP80, [peer(pod=POD("c"))])])],
         [("new", "Connected"), ("expect", "x/a", "x/c", "Dropped")], ("reachability", 1373, 1374)),
    step("GRP Pods X/B - update", [grp("x", "grp-pods-xa-then-xb", pod=POD("b"))],
         [("new", "Connected"), ("expect", "x/b", "x/c", "Dropped")], ("updatedReachability", 1376, 1377))]))

# ---------------------------------------------------------------------------------------- :1540 (Group Service refs)
CASES.append(case("ANNP Group Service Reference create and update", "testANNPGroupServiceRefCreateAndUpdate", steps=[
    step("Port 80", [svc("x", "svc1", {"app": "a"}), svc("x", "svc2", {"app": "b"}),
                     grp("x", "grp-svc1", service=["x", "svc1"]), grp("x", "grp-svc2", service=["x", "svc2"]),
                     annp("x", "annp-grp-svc-ref", 1.0, [at(group="grp-svc1")],
                          ingress=[rule("Drop", TCP80, [peer(group="grp-svc2")])])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped")], ("reachability", 1556, 1557)),
    step("Port 80 updated", [svc("x", "svc1", {"app": "b"}), svc("x", "svc3", {"app": "c"}),
                             grp("x", "grp-svc1", service=["x", "svc1"]), grp("x", "grp-svc2", service=["x", "svc3"])],
         [("new", "Connected"), ("expect", "x/c", "x/b", "Dropped")], ("reachability2", 1572, 1573))]))

# ---------------------------------------------------------------------------------------- :1439, :1489 (Service refs)
# testANNPGroupServiceRefPodAdd also probes two Pods it creates (CustomProbes: an app=b client to an
# app=a server, Dropped); the fixed 9-Pod universe does not model created Pods, so its allPods
# matrix is the step checked here.
_svcref = [svc("x", "svc1", {"app": "a"}), svc("x", "svc2", {"app": "b"}),
           grp("x", "grp-svc1", service=["x", "svc1"]), grp("x", "grp-svc2", service=["x", "svc2"]),
           annp("x", "annp-grp-svc-ref", 1.0, [at(group="grp-svc1")], ingress=[rule("Drop", TCP80, [peer(group="grp-svc2")])])]
CASES.append(case("ANNP Group Service Reference add pod", "testANNPGroupServiceRefPodAdd", steps=[
    step("Port 80 updated", _svcref, [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped")],
         ("reachability", 1471, 1472))]))
CASES.append(case("ANNP Group Service Reference delete", "testANNPGroupServiceRefDelete", steps=[
    step("Port 80", _svcref, [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped")], ("reachability", 1517, 1518)),
    step("Services deleted", [], [("new", "Connected")], ("reachability2", 1529, 1529),
         delete=[["Service", "svc1", "x"], ["Service", "svc2", "x"]])]))

# ---------------------------------------------------------------------------------------- :1589 (Group ipBlocks)
CASES.append(case("ANNP Drop Ingress From Group with ipBlocks to Pod: x/a", "testANNPGroupRefRuleIPBlocks", steps=[
    step("Port 80", [annp("x", "annp-deny-xb-xc-ips-ingress-for-xa", 1.0, [at(pod=POD("a"))],
                          ingress=[rule("Drop", TCP80, [peer(group="grp-ipblocks-pod-xb-xc")])]),
                     grp("x", "grp-ipblocks-pod-xb-xc", ipblocks=[{"cidr": "@x/b/32"}, {"cidr": "@x/c/32"}])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("expect", "x/c", "x/a", "Dropped")],
         ("reachability", 1610, 1612))]))

# ---------------------------------------------------------------------------------------- :1628 (nested Group)
CASES.append(case("ANNP nested Group create and update", "testANNPNestedGroupCreateAndUpdate", steps=[
    step("Port 80", [annp("x", "annp-nested-grp", 1.0, [at()], ingress=[rule("Drop", TCP80, [peer(group="grp-nested")])]),
                     svc("x", "svc1", {"app": "a"}), grp("x", "grp-svc-x-a", service=["x", "svc1"]),
                     grp("x", "grp-nested", children=["grp-svc-x-a", "grp-select-x-c"])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "x", "Dropped"), ("self", "Connected")],
         ("reachability", 1651, 1653)),
    step("Port 80 updated", [grp("x", "grp-select-x-b", pod=POD("b")),
                             grp("x", "grp-nested", children=["grp-svc-x-a", "grp-select-x-b", "grp-select-x-c"])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "x", "Dropped"), ("egress_to_ns", "x/b", "x", "Dropped"),
          ("self", "Connected")], ("reachability2", 1667, 1670)),
    step("Port 80 updated 2", [grp("x", "grp-select-x-c", pod=POD("c"))],
         [("new", "Connected"), ("egress_to_ns", "x/a", "x", "Dropped"), ("egress_to_ns", "x/b", "x", "Dropped"),
          ("egress_to_ns", "x/c", "x", "Dropped"), ("self", "Connected")], ("reachability3", 1697, 1701))]))

# ---------------------------------------------------------------------------------------- :1719 baseline tier (+ eval)
_baseline = acnp("acnp-baseline-isolate-ns-x", 1.0, [at(ns=NS("x"))], tier="baseline",
                 ingress=[rule("Drop", TCP80, [peer(ns={"labels": {}, "exprs": [["ns", "NotIn", ["x"]]]})])])
CASES.append(case("ACNP baseline tier namespace isolation", "testBaselineNamespaceIsolation", steps=[
    step("Baseline ACNP", [_baseline],
         [("new", "Connected"), ("ns_ingress_from_ns", "x", "y", "Dropped"), ("ns_ingress_from_ns", "x", "z", "Dropped")],
         ("reachability", 1734, 1736),
         evaluation=[("y/a", "x/a", "acnp-baseline-isolate-ns-x", "Drop"), ("y/b", "x/a", "acnp-baseline-isolate-ns-x", "Drop"),
                     ("z/a", "x/a", "acnp-baseline-isolate-ns-x", "Drop"), ("x/b", "x/a", "<NONE>", "<NONE>"),
                     ("z/b", "y/b", "<NONE>", "<NONE>")], eval_src=("evaluation", 1738, 1743)),
    step("Baseline ACNP with KNP", [_baseline, knp("x", "allow-y-a-to-x-a", POD("a"), ["Ingress"],
                                                   ingress=[{"ports": TCP80, "peers": [kpeer(pod=POD("a"), ns=NS("y"))]}])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("expect", "x/c", "x/a", "Dropped"),
          ("expect", "y/a", "x/b", "Dropped"), ("expect", "y/a", "x/c", "Dropped"), ("egress_to_ns", "y/b", "x", "Dropped"),
          ("egress_to_ns", "y/c", "x", "Dropped"), ("ns_ingress_from_ns", "x", "z", "Dropped")],
         ("reachabilityUpdated", 1755, 1762),
         evaluation=[("y/a", "x/a", "allow-y-a-to-x-a", "Allow"), ("y/b", "x/a", "allow-y-a-to-x-a", "Isolate"),
                     ("z/a", "x/a", "allow-y-a-to-x-a", "Isolate"), ("x/b", "x/a", "allow-y-a-to-x-a", "Isolate"),
                     ("z/b", "y/b", "<NONE>", "<NONE>")], eval_src=("evaluationUpdated", 1764, 1769))]))

# ---------------------------------------------------------------------------------------- :1800 priority override (+ eval)
_pr1 = acnp("acnp-priority1", 1.001, [at(pod=POD("a"), ns=NS("x"))], ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("z"))])])
_pr2 = acnp("acnp-priority2", 1.002, [at(pod=POD("a"), ns=NS("x"))], ingress=[rule("Allow", TCP80, [peer(ns=NS("z"))])])
_pr3 = acnp("acnp-priority3", 1.003, [at(ns=NS("x"))], ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])])
_two = [("new", "Connected")] + [("expect", "z/%s" % s, "x/%s" % d, "Dropped") for s in "abc" for d in "bc"]
_all = [("new", "Connected"), ("expect", "z/a", "x/b", "Dropped"), ("expect", "z/a", "x/c", "Dropped"),
        ("expect", "z/b", "x/a", "Dropped"), ("expect", "z/b", "x/b", "Dropped"), ("expect", "z/b", "x/c", "Dropped"),
        ("expect", "z/c", "x/b", "Dropped"), ("expect", "z/c", "x/c", "Dropped")]
CASES.append(case("ACNP PriorityOverride Intermediate", "testACNPPriorityOverride", steps=[
    step("Two Policies with different priorities", [_pr3, _pr2], _two, ("reachabilityTwoACNPs", 1825, 1831),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/b", "x/a", "acnp-priority2", "Allow"),
                     ("z/b", "x/b", "acnp-priority3", "Drop")], eval_src=("evaluationTwoACNPs", 1842, 1845))]))
CASES.append(case("ACNP PriorityOverride All", "testACNPPriorityOverride", steps=[
    step("All three Policies", [_pr3, _pr1, _pr2], _all, ("reachabilityAllACNPs", 1833, 1840),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/a", "x/a", "acnp-priority2", "Allow"),
                     ("z/a", "x/b", "acnp-priority3", "Drop"), ("z/b", "x/a", "acnp-priority1", "Drop")],
         eval_src=("evaluationAllACNPs", 1847, 1851))]))

# ---------------------------------------------------------------------------------------- :1883 tier override (+ eval)
_t1 = acnp("acnp-tier-emergency", 100, [at(pod=POD("a"), ns=NS("x"))], tier="emergency",
           ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("z"))])])
_t2 = acnp("acnp-tier-securityops", 10, [at(pod=POD("a"), ns=NS("x"))], tier="securityops",
           ingress=[rule("Allow", TCP80, [peer(ns=NS("z"))])])
_t3 = acnp("acnp-tier-application", 1, [at(ns=NS("x"))], tier="application", ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])])
CASES.append(case("ACNP TierOverride Intermediate", "testACNPTierOverride", steps=[
    step("Two Policies in different tiers", [_t3, _t2], _two, ("reachabilityTwoACNPs", 1911, 1917),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/b", "x/a", "acnp-tier-securityops", "Allow"),
                     ("z/b", "x/b", "acnp-tier-application", "Drop")], eval_src=("evaluationTwoACNPs", 1928, 1931))]))
CASES.append(case("ACNP TierOverride All", "testACNPTierOverride", steps=[
    step("All three Policies in different tiers", [_t3, _t1, _t2], _all, ("reachabilityAllACNPs", 1919, 1926),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/a", "x/a", "acnp-tier-securityops", "Allow"),
                     ("z/a", "x/b", "acnp-tier-application", "Drop"), ("z/b", "x/a", "acnp-tier-emergency", "Drop")],
         eval_src=("evaluationAllACNPs", 1933, 1937))]))

# ---------------------------------------------------------------------------------------- :1968 custom tiers (+ eval)
CASES.append(case("ACNP Custom Tier priority", "testACNPCustomTiers", steps=[
    step("Two Policies in different tiers",
         [{"kind": "Tier", "name": "high-priority", "priority": 245}, {"kind": "Tier", "name": "low-priority", "priority": 246},
          acnp("acnp-tier-low", 1, [at(ns=NS("x"))], tier="low-priority", ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])]),
          acnp("acnp-tier-high", 100, [at(pod=POD("a"), ns=NS("x"))], tier="high-priority",
               ingress=[rule("Allow", TCP80, [peer(ns=NS("z"))])])],
         _two, ("reachabilityTwoACNPs", 1995, 2001),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/b", "x/a", "acnp-tier-high", "Allow"),
                     ("z/b", "x/b", "acnp-tier-low", "Drop")], eval_src=("evaluationTwoACNPs", 2003, 2006))]))

# ---------------------------------------------------------------------------------------- :2030 / :2074 (+ eval)
CASES.append(case("ACNP Priority Conflicting Rule", "testACNPPriorityConflictingRule", steps=[
    step("Both ACNP", [acnp("acnp-drop", 1, [at(ns=NS("x"))], ingress=[rule("Drop", TCP80, [peer(ns=NS("z"))])]),
                       acnp("acnp-allow", 2, [at(ns=NS("x"))], ingress=[rule("Allow", TCP80, [peer(ns=NS("z"))])])],
         [("new", "Connected"), ("egress_to_ns", "z/a", "x", "Dropped"), ("egress_to_ns", "z/b", "x", "Dropped"),
          ("egress_to_ns", "z/c", "x", "Dropped")], ("reachabilityBothACNP", 2047, 2050),
         evaluation=[("y/a", "x/a", "<NONE>", "<NONE>"), ("z/a", "x/a", "acnp-drop", "Drop")],
         eval_src=("evaluationBothACNPs", 2052, 2054))]))
CASES.append(case("ACNP Rule Priority", "testACNPRulePriority", steps=[
    step("Both ACNP", [acnp("acnp-allow", 5, [at(ns=NS("x"))], egress=[rule("Allow", TCP80, [peer(ns=NS("z"))]),
                                                                       rule("Allow", TCP80, [peer(ns=NS("y"))])]),
                       acnp("acnp-deny", 5, [at(ns=NS("x"))], egress=[rule("Drop", TCP80, [peer(ns=NS("y"))]),
                                                                      rule("Drop", TCP80, [peer(ns=NS("z"))])])],
         [("new", "Connected"), ("ingress_from_ns", "y/a", "x", "Dropped"), ("ingress_from_ns", "y/b", "x", "Dropped"),
          ("ingress_from_ns", "y/c", "x", "Dropped")], ("reachabilityBothACNP", 2098, 2101),
         evaluation=[("x/b", "x/a", "<NONE>", "<NONE>"), ("x/a", "y/a", "acnp-deny", "Drop"),
                     ("x/a", "z/a", "acnp-allow", "Allow")], eval_src=("evaluationBothACNPs", 2103, 2106))]))

# ---------------------------------------------------------------------------------------- :2125 port range
CASES.append(case("ACNP Drop Egress From All Pod:a to NS:z with a portRange", "testACNPPortRange", steps=[
    step("ACNP Drop Ports 8080:8082", [acnp("acnp-deny-a-to-z-egress-port-range", 1.0, [at(pod=POD("a"))],
                                            egress=[rule("Drop", [port(8080, end=8082)], [peer(ns=NS("z"))],
                                                         name="acnp-port-range")])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/a", "z", "Dropped"),
          ("expect", "z/a", "z/b", "Dropped"), ("expect", "z/a", "z/c", "Dropped")], ("reachability", 2133, 2137),
         ports=(8080, 8081, 8082))]))

# ---------------------------------------------------------------------------------------- :2155 / :2190 Reject
CASES.append(case("ACNP Reject egress From All Pod:a to NS:z", "testACNPRejectEgress", steps=[
    step("Port 80", [acnp("acnp-reject-a-to-z-egress", 1.0, [at(pod=POD("a"))],
                          egress=[rule("Reject", TCP80, [peer(ns=NS("z"))])])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Rejected"), ("egress_to_ns", "y/a", "z", "Rejected"),
          ("expect", "z/a", "z/b", "Rejected"), ("expect", "z/a", "z/c", "Rejected")], ("reachability", 2163, 2167),
         evaluation=[("x/b", "z/a", "<NONE>", "<NONE>"), ("x/a", "z/a", "acnp-reject-a-to-z-egress", "Reject")],
         eval_src=("evaluation", 2169, 2171))]))
for _proto in ("TCP", "UDP"):
    CASES.append(case("ACNP Reject ingress from NS:z to All Pod:a " + _proto, "testACNPRejectIngress", steps=[
        step("Port 80", [acnp("acnp-reject-a-from-z-ingress", 1.0, [at(pod=POD("a"))],
                              ingress=[rule("Reject", [port(80, _proto)], [peer(ns=NS("z"))])])],
             [("new", "Connected"), ("ingress_from_ns", "x/a", "z", "Rejected"), ("ingress_from_ns", "y/a", "z", "Rejected"),
              ("expect", "z/b", "z/a", "Rejected"), ("expect", "z/c", "z/a", "Rejected")], ("reachability", 2198, 2202),
             protocol=_proto)]))

# ---------------------------------------------------------------------------------------- :2413 / :2441 ANNP
CASES.append(case("ANNP Drop Egress y/b to x/c with a portRange", "testANNPPortRange", steps=[
    step("ANNP Drop Ports 8080:8082", [annp("y", "annp-deny-yb-to-xc-egress-port-range", 1.0, [at(pod=POD("b"))],
                                            egress=[rule("Drop", [port(8080, end=8082)], [peer(pod=POD("c"), ns=NS("x"))],
                                                         name="annp-port-range")])],
         [("new", "Connected"), ("expect", "y/b", "x/c", "Dropped")], ("reachability", 2421, 2422),
         ports=(8080, 8081, 8082))]))
_annp_basic = annp("y", "np-same-name", 1.0, [at(pod=POD("a"))], ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))])])
CASES.append(case("ANNP Drop X/B to Y/A", "testANNPBasic", steps=[
    step("Port 80", [_annp_basic], [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped")], ("reachability", 2449, 2450))]))
CASES.append(case("With K8s NetworkPolicy of the same name", "testANNPBasic", steps=[
    step("Port 80", [_annp_basic, knp("y", "np-same-name", POD("a"), [], ingress=[{"ports": TCP80, "peers": []}])],
         [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped")], ("reachability", 2449, 2450))]))

# ---------------------------------------------------------------------------------------- :2484 ANNP update (+ eval)
CASES.append(case("ANNP update", "testANNPUpdate", steps=[
    step("Drop", [annp("y", "np-update", 1.0, [at(pod=POD("a"))], ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped")], ("reachability", 2492, 2493),
         evaluation=[("x/a", "y/a", "<NONE>", "<NONE>"), ("x/b", "y/a", "np-update", "Drop")], eval_src=("evaluation", 2494, 2496)),
    step("Allow", [annp("y", "np-update", 1.0, [at(pod=POD("a"))], ingress=[rule("Allow", TCP80, [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Connected")], ("updatedReachability", 2516, 2516),
         evaluation=[("x/a", "y/a", "<NONE>", "<NONE>"), ("x/b", "y/a", "np-update", "Allow")],
         eval_src=("updatedEvaluation", 2517, 2519))]))

# ---------------------------------------------------------------------------------------- :2539 multiple appliedTo (+ eval)
_TMP = "temp-e2e"
for _single in (True, False):
    if _single:
        _mat = annp("y", "np-multiple-appliedto", 1.0, [at(pod=POD("a")), at(pod={"labels": {_TMP: ""}})],
                    ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))])])
    else:
        _mat = annp("y", "np-multiple-appliedto", 1.0, None,
                    ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))], at=[at(pod=POD("a"))]),
                             rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))], at=[at(pod={"labels": {_TMP: ""}})])])
    CASES.append(case("ANNP multiple appliedTo " + ("single rule" if _single else "multiple rules"),
                      "testANNPMultipleAppliedTo", steps=[
        step("Drop x/b to y/a", [_mat], [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped")], ("reachability", 2556, 2557),
             evaluation=[("x/b", "y/c", "<NONE>", "<NONE>"), ("x/b", "y/a", "np-multiple-appliedto", "Drop")],
             eval_src=("evaluation", 2558, 2560)),
        step("y/c labelled", [{"kind": "PodLabels", "name": "y/c", "labels": {"pod": "c", "app": "c", _TMP: ""}}],
             [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped"), ("expect", "x/b", "y/c", "Dropped")],
             ("reachability", 2583, 2585),
             evaluation=[("x/b", "y/c", "np-multiple-appliedto", "Drop"), ("x/b", "y/a", "np-multiple-appliedto", "Drop")],
             eval_src=("updatedEvaluation", 2586, 2588)),
        step("y/c unlabelled", [{"kind": "PodLabels", "name": "y/c", "labels": {"pod": "c", "app": "c"}}],
             [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped")], ("reachability", 2604, 2605),
             evaluation=[("x/b", "y/c", "<NONE>", "<NONE>"), ("x/b", "y/a", "np-multiple-appliedto", "Drop")],
             eval_src=("evaluation", 2558, 2560))]))

# ---------------------------------------------------------------------------------------- :2901 appliedTo per rule
CASES.append(case("ANNP AppliedTo per rule", "testAppliedToPerRule", steps=[
    step("Port 80", [annp("y", "np1", 1.0, None,
                          ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))], at=[at(pod=POD("a"))]),
                                   rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("z"))], at=[at(pod=POD("b"))])])],
         [("new", "Connected"), ("expect", "x/b", "y/a", "Dropped"), ("expect", "z/b", "y/b", "Dropped")],
         ("reachability", 2911, 2913))]))
CASES.append(case("ACNP AppliedTo per rule", "testAppliedToPerRule", steps=[
    step("Port 80", [acnp("cnp1", 1.0, None,
                          ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("x"))], at=[at(pod=POD("a"))]),
                                   rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("z"))], at=[at(pod=POD("b"), ns=NS("y"))])])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("expect", "x/b", "y/a", "Dropped"),
          ("expect", "x/b", "z/a", "Dropped"), ("expect", "z/b", "y/b", "Dropped")], ("reachability2", 2935, 2939))]))

# ---------------------------------------------------------------------------------------- :2956 CG Service refs
_cgsvc = acnp("cnp-cg-svc-ref", 1.0, [at(group="cg-svc1")], ingress=[rule("Drop", TCP80, [peer(group="cg-svc2")])])
CASES.append(case("ACNP ClusterGroup Service Reference create and update", "testACNPClusterGroupServiceRefCreateAndUpdate", steps=[
    step("Port 80", [svc("x", "svc1", {"app": "a"}), svc("y", "svc2", {"app": "b"}), cg("cg-svc1", service=["x", "svc1"]),
                     cg("cg-svc2", service=["y", "svc2"]), _cgsvc],
         [("new", "Connected"), ("expect", "y/b", "x/a", "Dropped")], ("reachability", 2972, 2973)),
    step("Port 80 updated", [svc("x", "svc1", {"app": "b"}), svc("y", "svc3", {"app": "a"}), cg("cg-svc1", service=["x", "svc1"]),
                             cg("cg-svc2", service=["y", "svc3"])],
         [("new", "Connected"), ("expect", "y/a", "x/b", "Dropped")], ("reachability2", 3004, 3005)),
    step("Port 80 ACNP spec updated to selector",
         [acnp("cnp-cg-svc-ref", 1.0, [at(pod=POD("a"), ns=NS("x"))], ingress=[rule("Drop", TCP80, [peer(pod=POD("b"), ns=NS("y"))])])],
         [("new", "Connected"), ("expect", "y/b", "x/a", "Dropped")], ("reachability", 2972, 2973))]))

# ---------------------------------------------------------------------------------------- :3037 nested CG
CASES.append(case("ACNP nested ClusterGroup create and update", "testACNPNestedClusterGroupCreateAndUpdate", steps=[
    step("Port 80", [acnp("cnp-nested-cg", 1.0, [at(ns=NS("z"))], ingress=[rule("Drop", TCP80, [peer(group="cg-nested")])]),
                     svc("x", "svc1", {"app": "a"}), cg("cg-svc-x-a", service=["x", "svc1"]),
                     cg("cg-nested", children=["cg-svc-x-a", "cg-select-y-c"])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped")], ("reachability", 3064, 3065)),
    step("Port 80 updated", [cg("cg-select-y-b", pod=POD("b"), ns=NS("y")),
                             cg("cg-nested", children=["cg-svc-x-a", "cg-select-y-b", "cg-select-y-c"])],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/b", "z", "Dropped")],
         ("reachability2", 3079, 3081)),
    step("Port 80 updated 2", [cg("cg-select-y-c", pod=POD("c"), ns=NS("y"))],
         [("new", "Connected"), ("egress_to_ns", "x/a", "z", "Dropped"), ("egress_to_ns", "y/b", "z", "Dropped"),
          ("egress_to_ns", "y/c", "z", "Dropped")], ("reachability3", 3108, 3111))]))

# ---------------------------------------------------------------------------------------- :3127 nested ipBlock CG
CASES.append(case("ACNP Drop Ingress From x to Pod y/a with nested ClusterGroup with ipBlocks",
                  "testACNPNestedIPBlockClusterGroupCreateAndUpdate", steps=[
    step("Port 80", [acnp("acnp-deny-x-ips-ingress-for-ya", 1.0, [at(pod=POD("a"), ns=NS("y"))],
                          ingress=[rule("Drop", TCP80, [peer(group="cg-parent")])]),
                     cg("cg-x-a-ipb", ipblocks=[{"cidr": "@x/a/32"}]), cg("cg-x-b-ipb", ipblocks=[{"cidr": "@x/b/32"}]),
                     cg("cg-parent", children=["cg-x-a-ipb", "cg-x-b-ipb"])],
         [("new", "Connected"), ("expect", "x/a", "y/a", "Dropped"), ("expect", "x/b", "y/a", "Dropped")],
         ("reachability", 3156, 3158)),
    step("Port 80, updated", [cg("cg-select-x-c", pod=POD("c"), ns=NS("x")), cg("cg-parent", children=["cg-x-a-ipb", "cg-select-x-c"])],
         [("new", "Connected"), ("expect", "x/a", "y/a", "Dropped"), ("expect", "x/c", "y/a", "Dropped")],
         ("reachability2", 3174, 3176))]))

# ---------------------------------------------------------------------------------------- :3191 namespace isolation
CASES.append(case("ACNP Namespace isolation for all namespaces", "testACNPNamespaceIsolation", steps=[
    step("Port 80", [acnp("test-acnp-ns-isolation", 1.0, [at(ns=ALL)], tier="baseline",
                          ingress=[rule("Allow", None, [peer(ns_match="Self")]), rule("Drop", None, [peer(ns=ALL)])])],
         [("new", "Dropped"), ("all_self_ns", "Connected")], ("reachability", 3203, 3204))]))
CASES.append(case("ACNP Namespace isolation for namespace x", "testACNPNamespaceIsolation", steps=[
    step("Port 80", [acnp("test-acnp-ns-isolation-applied-to-per-rule", 1.0, None, tier="baseline",
                          egress=[rule("Allow", None, [peer(ns_match="Self")], at=[at(ns=NS("x"))]),
                                  rule("Drop", None, [peer(ns=ALL)], at=[at(ns=NS("x"))])])],
         [("new", "Connected")] + [("egress_to_ns", "x/%s" % p, n, "Dropped") for p in "abc" for n in "yz"],
         ("reachability2", 3222, 3228))]))

# ---------------------------------------------------------------------------------------- :3244 strict isolation (Pass)
_strict = acnp("test-acnp-strict-ns-isolation", 1.0, [at(ns=ALL)], tier="securityops",
               ingress=[rule("Pass", None, [peer(ns_match="Self")]), rule("Drop", None, [peer(ns=ALL)])])
CASES.append(case("ACNP strict Namespace isolation for all Namespaces", "testACNPStrictNamespacesIsolation", steps=[
    step("Namespace isolation, Port 80", [_strict], [("new", "Dropped"), ("all_self_ns", "Connected")],
         ("reachability", 3256, 3257)),
    step("Namespace isolation with K8s NP, Port 80", [knp("x", "default-deny-in-namespace-x", {}, ["Ingress"])],
         [("new", "Dropped"), ("all_self_ns", "Connected"), ("self_ns", "x", "Dropped"), ("self", "Connected")],
         ("reachability2", 3270, 3273))]))

# ---------------------------------------------------------------------------------------- :3288 / :3332 sameLabels
_EXT = {"prod1": {"purpose": "test", "tier": "prod"}, "prod2": {"purpose": "test", "tier": "prod"},
        "dev1": {"purpose": "test", "tier": "dev"}, "dev2": {"purpose": "test", "tier": "dev"},
        "no-tier": {"purpose": "test-exclusion"}}
CASES.append(case("ACNP strict Namespace isolation by Namespace purpose and tier labels",
                  "testACNPStrictNamespacesIsolationByLabels", universe=_EXT, steps=[
    step("Namespace isolation by label, Port 80",
         [acnp("test-acnp-strict-ns-isolation-by-labels", 1.0, [at(ns=ALL)], tier="securityops",
               ingress=[rule("Pass", None, [peer(ns_match={"same_labels": ["purpose", "tier"]})]),
                        rule("Drop", None, [peer(ns=ALL)])])],
         [("new", "Dropped"), ("ns_ingress_from_ns", "prod1", "prod2", "Connected"),
          ("ns_egress_to_ns", "prod1", "prod2", "Connected"), ("ns_ingress_from_ns", "prod2", "prod1", "Connected"),
          ("ns_egress_to_ns", "prod2", "prod1", "Connected"), ("ns_ingress_from_ns", "dev1", "dev2", "Connected"),
          ("ns_egress_to_ns", "dev1", "dev2", "Connected"), ("ns_ingress_from_ns", "dev2", "dev1", "Connected"),
          ("ns_egress_to_ns", "dev2", "dev1", "Connected"), ("all_self_ns", "Connected"), ("self_ns", "no-tier", "Dropped"),
          ("self", "Connected")], ("reachability", 3306, 3317))]))
CASES.append(case("ACNP strict Namespace isolation by single purpose label",
                  "testACNPStrictNamespacesIsolationBySingleLabel", universe=_EXT, steps=[
    step("Namespace isolation by single label, Port 80",
         [acnp("test-acnp-strict-ns-isolation-by-single-purpose-label", 1.0, [at(ns=ALL)], tier="securityops",
               ingress=[rule("Pass", None, [peer(ns_match={"same_labels": ["purpose"]})]), rule("Drop", None, [peer(ns=ALL)])])],
         [("new", "Connected")] + [("ns_egress_to_ns", n, "no-tier", "Dropped") for n in ("prod1", "prod2", "dev1", "dev2")] +
         [("ns_ingress_from_ns", n, "no-tier", "Dropped") for n in ("prod1", "prod2", "dev1", "dev2")],
         ("reachability", 3347, 3355))]))

# ---------------------------------------------------------------------------------------- :446 source ports
_SP = dict(sport=32768, send=60999)  # getTCPv4SourcePortRangeFromPod: the Linux default ephemeral range
CASES.append(case("ACNP Drop X/B to A based on source port", "testACNPSourcePort", steps=[
    step("Port 80", [acnp("acnp-source-port", 1.0, [at(pod=POD("a"))],
                          ingress=[rule("Drop", [port(None, **_SP)], [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("expect", "x/b", "y/a", "Dropped"),
          ("expect", "x/b", "z/a", "Dropped")], ("reachability", 470, 473)),
    step("Port 81", [acnp("acnp-source-port", 1.0, [at(pod=POD("a"))],
                          ingress=[rule("Drop", [port(80, **_SP)], [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Connected")], ("updatedReachability", 475, 475), ports=(81,)),
    step("Port range 80-81", [acnp("acnp-source-port", 1.0, [at(pod=POD("a"))],
                                   ingress=[rule("Drop", [port(80, end=81, **_SP)], [peer(pod=POD("b"), ns=NS("x"))])])],
         [("new", "Connected"), ("expect", "x/b", "x/a", "Dropped"), ("expect", "x/b", "y/a", "Dropped"),
          ("expect", "x/b", "z/a", "Dropped")], ("reachability", 470, 473), ports=(80, 81))]))

# ---------------------------------------------------------------------------------------- networkpolicy_test.go
# The K8s NetworkPolicy suite probes single client -> server pairs (runNetcatCommandFromTestPod); its Pods
# carry the label antrea-e2e=<name> in the test Namespace. Expectations are the Fatalf conditions.
_NPU = {"namespaces": {"testns": {}}, "pods": [["testns", "client", {"antrea-e2e": "client"}],
                                               ["testns", "server-a", {"antrea-e2e": "server-a", "app": "nginx"}],
                                               ["testns", "server-b", {"antrea-e2e": "server-b", "app": "nginx"}]]}
_NPU6 = dict(_NPU, family=6)


def probe(src, dst, mark, port_=80):
    return ("probe", src, dst, port_, mark)


CASES.append(case("K8s NP default deny egress", "testDefaultDenyEgressPolicy", go_file=GO_NP, universe=_NPU, steps=[
    step("before", [], [probe("testns/client", "testns/server-a", "Connected")], ("preCheckFunc", 426, 430)),
    step("deny-all-egress", [knp("testns", "test-networkpolicy-deny-all-egress", {}, ["Egress"], egress=[])],
         [probe("testns/client", "testns/server-a", "Dropped")], ("npCheck", 453, 457))]))
CASES.append(case("K8s NP egress to server in CIDR block (IPv6)", "testEgressToServerInCIDRBlock", go_file=GO_NP, universe=_NPU6,
                  steps=[
    step("before", [], [probe("testns/client", "testns/server-a", "Connected"),
                        probe("testns/client", "testns/server-b", "Connected")], ("runNetcat", 490, 495)),
    step("allow /128", [knp("testns", "allow-client-a-via-cidr-egress-rule", S(**{"antrea-e2e": "client"}), ["Egress"],
                            egress=[{"ports": None, "peers": [kpeer(cidr="@testns/server-a/128")]}])],
         [probe("testns/client", "testns/server-a", "Connected"), probe("testns/client", "testns/server-b", "Dropped")],
         ("runNetcat", 526, 531))]))
CASES.append(case("K8s NP egress to server in CIDR block with exception (IPv6)", "testEgressToServerInCIDRBlockWithException",
                  go_file=GO_NP, universe=_NPU6, steps=[
    step("deny via except", [knp("testns", "deny-client-a-via-except-cidr-egress-rule", S(**{"antrea-e2e": "client"}), ["Egress"],
                                 egress=[{"ports": None, "peers": [kpeer(cidr="fd00:10::/64", except_=["@testns/server-a/128"])]}])],
         [probe("testns/client", "testns/server-a", "Dropped")], ("runNetcat", 594, 596))]))
