"""CPU tier, property-based: small random NetworkPolicy rule sets over a tiny address / port
universe (so rules overlap, share conjunctive match flows, tie in priority and hit each other's
packets), checked three ways -- the product compiler's flow dump equals the oracle compiler's,
and the product image evaluated by the host emulation of the kernel body (tests/csrc/emu.cpp,
same core.hpp as the device) gives the Python OVS oracle's verdict for every packet of a random
batch drawn from the same universe. hypothesis shrinks a failure to a minimal rule set."""
import copy

import numpy as np
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from antrea_amd import gpc  # noqa: E402
from tests.test_emu_parity import _cmp, oracle_verdicts, product_verdicts  # noqa: E402
from tests.util import assign_tables, normalize_flows  # noqa: E402

IPS = ["10.0.0.%d" % i for i in range(8)]
CIDRS = ["10.0.0.0/29", "10.0.0.4/30", "10.0.0.0/24", "10.0.1.0/24", "0.0.0.0/0"]
PORTS = [80, 81, 443, 1000, 5000]

addr = st.one_of(st.sampled_from(IPS), st.sampled_from(CIDRS))
ofport = st.builds(lambda p: {"ofport": p}, st.integers(1, 4))


def _svc():
    l4 = st.builds(lambda proto, port, width: {"protocol": proto, "port": port, **({"end_port": port + width}
                                                                                  if width else {})},
                   st.sampled_from(["TCP", "UDP"]), st.sampled_from(PORTS), st.sampled_from([0, 0, 1, 7]))
    icmp = st.builds(lambda t: {"protocol": "ICMP", "icmp_type": t, "icmp_code": 0}, st.sampled_from([0, 8]))
    proto_only = st.builds(lambda p: {"protocol": p}, st.sampled_from(["TCP", "UDP"]))
    return st.one_of(st.none(), st.lists(st.one_of(l4, icmp, proto_only), min_size=0, max_size=2))


@st.composite
def rule(draw, fid):
    k8s = draw(st.booleans())
    direction = draw(st.sampled_from(["In", "Out"]))
    peers = st.one_of(st.none(), st.lists(addr, min_size=0, max_size=3))
    applied = st.lists(ofport if direction == "In" else st.sampled_from(IPS[:4]), min_size=1, max_size=2)
    r = {"direction": direction, "flow_id": fid, "name": "r%d" % fid,
         "policy_type": "K8sNetworkPolicy" if k8s else "AntreaClusterNetworkPolicy",
         "policy_namespace": "" if not k8s else "ns", "policy_name": "p%d" % fid, "policy_uid": "u%d" % fid,
         "service": draw(_svc()), "enable_logging": draw(st.sampled_from([False, False, True]))}
    if direction == "In":
        r["from"], r["to"] = draw(peers), draw(applied)
    else:
        r["from"], r["to"] = draw(applied), draw(peers)
    if not k8s:
        r["action"] = draw(st.sampled_from(["Allow", "Drop", "Reject", "Pass"]))
        r["priority"] = draw(st.sampled_from([100, 100, 101, 200]))  # equal priorities: ties
        r["tier_priority"] = draw(st.sampled_from([50, 250]))
    return r


@st.composite
def rule_set(draw):
    n = draw(st.integers(1, 6))
    return assign_tables([draw(rule(100 + i)) for i in range(n)])


@st.composite
def packets(draw):
    n = 48
    ip_pool = [int.from_bytes(bytes(map(int, a.split("."))), "big") for a in IPS] + [0x0A000109, 0x0B000001]
    pick = lambda: st.lists(st.sampled_from(ip_pool), min_size=n, max_size=n)
    proto = draw(st.lists(st.sampled_from([6, 6, 17, 1]), min_size=n, max_size=n))
    dport = draw(st.lists(st.sampled_from(PORTS + [1003, 1007, 1008]), min_size=n, max_size=n))
    icmp_t = draw(st.lists(st.sampled_from([0, 8]), min_size=n, max_size=n))
    return {"src": np.array(draw(pick()), np.uint32), "dst": np.array(draw(pick()), np.uint32),
            "sport": np.array([t if p == 1 else 40000 for t, p in zip(icmp_t, proto)], np.uint16),
            "dport": np.array([0 if p == 1 else d for d, p in zip(dport, proto)], np.uint16),
            "proto": np.array(proto, np.uint8),
            "out_port": np.array(draw(st.lists(st.integers(1, 4), min_size=n, max_size=n)), np.uint32),
            "ct_state": np.array(draw(st.lists(st.sampled_from([0x21, 0x21, 0x21, 0x22]), min_size=n,
                                               max_size=n)), np.uint8)}


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_EXAMPLES", "100")), deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(rules=rule_set(), cols=packets())
def test_random_rule_sets_product_equals_oracle(rules, cols):
    from oracle import compiler as oc
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(rules))
    got, c = product_verdicts(rules, cols)
    assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows())
    want, _ = oracle_verdicts(rules, cols, len(cols["src"]))
    _cmp(got, want, cols)
    # flow-text seam: the oracle's dump loaded as text classifies the same (tiers are
    # a PolicyRule attribute, not a flow field: compared without them)
    from tests import emu
    d = gpc.Classifier()
    loaded, skipped = d.load_flows(fnp.dump_flows())
    assert skipped == 0 and normalize_flows(d.dump_flows()) == normalize_flows(fnp.dump_flows())
    emu.commit_host(d)
    a, b = emu.classify(d, cols), want.copy()
    a["tier"] = 0
    b["tier"] = 0
    _cmp(a, b, cols)


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_EXAMPLES", "100")) // 2, deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(rules=rule_set(), cols=packets())
def test_random_rule_sets_plain_driver(rules, cols):
    """The same property without composite driver indexes (GPC_COMPOSITE=0: every table keeps the
    plain per-clause driver index; by default tables whose rules all hold a few exact AppliedTo
    values get the (band key, value) index of core.hpp TableHdr cidx)."""
    import os
    old = os.environ.get("GPC_COMPOSITE")
    os.environ["GPC_COMPOSITE"] = "0"
    try:
        got, _ = product_verdicts(rules, cols)
    finally:
        if old is None:
            del os.environ["GPC_COMPOSITE"]
        else:
            os.environ["GPC_COMPOSITE"] = old
    want, _ = oracle_verdicts(rules, cols, len(cols["src"]))
    _cmp(got, want, cols)


@st.composite
def churn(draw):
    """A rule set, then 1-8 control-plane operations on it (the agent's churn path, network_policy.go
    1570-1710, 1873), each published with gpc_commit (delta epochs on the product side)."""
    rules = draw(rule_set())
    ops = []
    for _ in range(draw(st.integers(1, 8))):
        i = draw(st.integers(0, len(rules) - 1))
        r = rules[i]
        kind = draw(st.sampled_from(["add", "add", "del", "uninstall", "reinstall", "reassign"]))
        side = draw(st.sampled_from(["src", "dst"]))
        peer_side = "dst" if r["direction"] == "Out" else "src"
        if side == peer_side:
            addrs = draw(st.lists(addr, min_size=1, max_size=2))
        elif r["direction"] == "In":
            addrs = draw(st.lists(ofport, min_size=1, max_size=2))
        else:
            addrs = draw(st.lists(st.sampled_from(IPS[:6]), min_size=1, max_size=2))
        ops.append((kind, i, side, addrs))
    return rules, ops


def _both(fnp, c, fn):
    """Apply one operation to the oracle and the product: both succeed or both fail."""
    errs = []
    for side in (fnp, c):
        try:
            fn(side)
            errs.append(None)
        except Exception as e:  # noqa: BLE001 -- the error class differs, the outcome must not
            errs.append(e)
    assert (errs[0] is None) == (errs[1] is None), errs
    return errs[1] is None


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_EXAMPLES", "100")), deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(case=churn(), cols=packets())
def test_random_churn_product_equals_oracle(case, cols):
    """Random churn in lock step: after every operation the realized flows are identical, and at the
    end the product's committed image (base + journal delta epochs, host emulation of the kernel
    body) gives the Python oracle's verdicts."""
    _churn_body(case, cols)


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_EXAMPLES", "100")) // 2, deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(case=churn(), cols=packets())
def test_random_churn_plain_driver(case, cols):
    """The churn property over base images without composite driver indexes (GPC_COMPOSITE=0;
    the default property runs over composite bases: delta epochs, tombstones, compaction)."""
    import os
    old = os.environ.get("GPC_COMPOSITE")
    os.environ["GPC_COMPOSITE"] = "0"
    try:
        _churn_body(case, cols)
    finally:
        if old is None:
            del os.environ["GPC_COMPOSITE"]
        else:
            os.environ["GPC_COMPOSITE"] = old


def _churn_body(case, cols):
    from oracle import compiler as oc
    from oracle import ovs_cls
    from tests import emu
    rules, ops = case
    rules = copy.deepcopy(rules)
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.initialize()
        side.batch_install_policy_rule_flows(copy.deepcopy(rules))
    emu.commit_host(c, full=True)
    installed = {r["flow_id"]: True for r in rules}
    for kind, i, side, addrs in ops:
        r = rules[i]
        fid, prio = r["flow_id"], r.get("priority")
        if kind == "add":
            _both(fnp, c, lambda s: s.add_policy_rule_address(fid, side, copy.deepcopy(addrs), prio))
        elif kind == "del":
            _both(fnp, c, lambda s: s.delete_policy_rule_address(fid, side, copy.deepcopy(addrs), prio))
        elif kind == "uninstall" and installed[fid]:
            if _both(fnp, c, lambda s: s.uninstall_policy_rule_flows(fid)):
                installed[fid] = False
        elif kind == "reinstall" and not installed[fid]:
            if _both(fnp, c, lambda s: s.install_policy_rule_flows(copy.deepcopy(r))):
                installed[fid] = True
        elif kind == "reassign" and prio is not None:
            upd = {prio: prio + 1000}
            if _both(fnp, c, lambda s: s.reassign_flow_priorities(upd, r["table"])):
                for q in rules:
                    if q.get("priority") == prio and q["table"] == r["table"]:
                        q["priority"] = prio + 1000
        assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows()), (kind, fid, side, addrs)
        emu.commit_host(c)
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in rules}
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), tiers)
    n = len(cols["src"])
    want = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for k in range(n):
        e, g = pipe.classify({key: int(v[k]) for key, v in cols.items()})
        for j, v in enumerate((e, g)):
            want[k, j] = (v[1], v[0], v[2], v[3], v[4])
    _, slots = c.counters()
    cnt = np.zeros((max(1, len(slots)), 3), np.uint64)
    _cmp(emu.classify(c, cols, counters=cnt), want, cols)
    per_conj = {int(s): tuple(int(x) for x in cnt[i]) for i, s in enumerate(slots) if s and cnt[i].any()}
    # a full rebuild (compaction) of the same state: same verdicts, same per-rule counts
    emu.commit_host(c, full=True)
    _, slots2 = c.counters()
    cnt2 = np.zeros((max(1, len(slots2)), 3), np.uint64)
    _cmp(emu.classify(c, cols, counters=cnt2), want, cols)
    assert per_conj == {int(s): tuple(int(x) for x in cnt2[i]) for i, s in enumerate(slots2) if s and cnt2[i].any()}
    # ... and the Metric-table counters of the C oracle over the oracle's flows (NetworkPolicyMetrics)
    from oracle import parity
    from oracle.cls_c import CPipeline
    cp = CPipeline(fnp.dump_flows(), tiers, procs=1)
    cp.classify(cols, threads=1, count=True)
    assert per_conj == {k: v for k, v in parity.oracle_metrics(cp).items() if any(v)}


IPS6 = ["fd00::%x" % i for i in range(1, 4)] + ["fd00::/126", "fd00::/64"]


@st.composite
def rich_rule(draw, fid):
    """rule() plus IPv6 peers (dual-stack flows), ANNP / BANP (baseline tier: *DefaultRule tables),
    logging, source-port ranges."""
    r = draw(rule(fid))
    kind = draw(st.sampled_from(["K8sNetworkPolicy", "AntreaClusterNetworkPolicy", "AntreaNetworkPolicy",
                                 "BaselineAdminNetworkPolicy"]))
    r["policy_type"] = kind
    if kind == "K8sNetworkPolicy":
        for k in ("action", "priority", "tier_priority"):
            r.pop(k, None)
    else:
        r.setdefault("action", draw(st.sampled_from(["Allow", "Drop", "Reject"])))
        r.setdefault("priority", draw(st.sampled_from([100, 101])))
        if kind == "BaselineAdminNetworkPolicy":
            r["action"] = draw(st.sampled_from(["Allow", "Drop"]))
            r["priority"] = draw(st.sampled_from([10, 11, 20]))
            r["table"] = "EgressDefaultRule" if r["direction"] == "Out" else "IngressDefaultRule"
    peer_key = "to" if r["direction"] == "Out" else "from"
    if r[peer_key] is not None and draw(st.booleans()):
        r[peer_key] = r[peer_key] + draw(st.lists(st.sampled_from(IPS6), min_size=1, max_size=2))
    if r["service"] and draw(st.booleans()):
        s = dict(r["service"][0])
        if s.get("protocol") in ("TCP", "UDP"):
            s.update(src_port=40000, src_end_port=40003)
            r["service"] = [s] + r["service"][1:]
    return r


@st.composite
def rich_packets(draw):
    cols = draw(packets())
    n = len(cols["src"])
    cols["ct_state"] = np.array(draw(st.lists(st.sampled_from([0x21, 0x21, 0x22, 0x24, 0x2a]), min_size=n,
                                              max_size=n)), np.uint8)
    cols["dest"] = np.array(draw(st.lists(st.sampled_from([0, 0, 0, 1, 2, 3]), min_size=n, max_size=n)), np.uint8)
    cols["ct_mark"] = np.array(draw(st.lists(st.sampled_from([0, 0, 0, 0x40]), min_size=n, max_size=n)), np.uint8)
    cols["sport"] = np.where(cols["proto"] == 1, cols["sport"],
                             np.array(draw(st.lists(st.sampled_from([40000, 40002, 40004]), min_size=n, max_size=n)),
                                      np.uint16)).astype(np.uint16)
    return cols


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_EXAMPLES", "100")), deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(rules=st.integers(1, 6).flatmap(lambda n: st.tuples(*[rich_rule(100 + i) for i in range(n)])),
       cols=rich_packets(), dns=st.booleans())
def test_random_dual_stack_rule_sets_product_equals_oracle(rules, cols, dns):
    """Dual-stack contexts (IPv4 + IPv6 flows), all policy kinds incl. the baseline tier, logging,
    source-port ranges, a DNS interception conjunction, and packets with conntrack states,
    IngressSecurityClassifier destinations and the hairpin mark: product == oracle flows, and the
    IPv4 verdicts of the emulated product image == the Python oracle's."""
    from oracle import compiler as oc
    from oracle import ovs_cls
    from tests import emu
    rules = assign_tables([copy.deepcopy(r) for r in rules])
    fnp, c = oc.FeatureNetworkPolicy(ipv4=True, ipv6=True), gpc.Classifier(ipv4=True, ipv6=True)
    for side in (fnp, c):
        side.initialize()
        if dns:
            side.new_dns_packet_in_conjunction(7)
            side.add_address_to_dns_conjunction(7, ["10.0.0.2", "fd00::2"])
        side.batch_install_policy_rule_flows(copy.deepcopy(rules))
    assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows())
    emu.commit_host(c)
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in rules}
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), tiers)
    n = len(cols["src"])
    want = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for k in range(n):
        e, g = pipe.classify({key: int(v[k]) for key, v in cols.items()})
        for j, v in enumerate((e, g)):
            want[k, j] = (v[1], v[0], v[2], v[3], v[4])
    _cmp(emu.classify(c, cols), want, cols)
    # IPv6 packets of the same batch (addresses from the IPv6 peers' universe) through the IPv6 image
    import ipaddress
    pool6 = [int(ipaddress.IPv6Address("fd00::%x" % i)) for i in range(1, 6)] + [int(ipaddress.IPv6Address("fe80::1"))]
    rng = np.random.default_rng(int(cols["src"][0]) ^ n)
    s6 = [pool6[k] for k in rng.integers(0, len(pool6), n)]
    d6 = [pool6[k] for k in rng.integers(0, len(pool6), n)]
    cols6 = {k: v for k, v in cols.items() if k not in ("src", "dst")}
    cols6["proto"] = np.where(cols["proto"] == 1, 58, cols["proto"]).astype(np.uint8)
    cols6["src6"] = np.array([list(x.to_bytes(16, "big")) for x in s6], np.uint8)
    cols6["dst6"] = np.array([list(x.to_bytes(16, "big")) for x in d6], np.uint8)
    want6 = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for k in range(n):
        pkt = {key: int(v[k]) for key, v in cols6.items() if v.ndim == 1}
        pkt.update(src=s6[k], dst=d6[k], eth=0x86DD)
        e, g = pipe.classify(pkt)
        for j, v in enumerate((e, g)):
            want6[k, j] = (v[1], v[0], v[2], v[3], v[4])
    _cmp(emu.classify6(c, cols6), want6, cols6)
    # the C restatement (the full-scale checker and CPU baseline) agrees with the Python one
    from oracle.cls_c import CPipeline
    cp = CPipeline(fnp.dump_flows(), tiers, procs=1)
    got_c = cp.classify(cols, threads=1)
    _cmp(np.ascontiguousarray(got_c).view(gpc.VERDICT_DTYPE).reshape(-1, 2), want, cols)


@settings(max_examples=int(__import__("os").environ.get("GPC_FUZZ_SVC_EXAMPLES", "15")), deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(1, 10_000), c1=st.booleans(), n_svc=st.integers(1, 40), eps=st.integers(1, 6))
def test_random_services_product_equals_oracle(seed, c1, n_svc, eps):
    """AntreaProxy stage on random Service sets (Endpoints local / remote, no-Endpoint
    Services, Local traffic policy) in front of random policies: the emulated product's verdicts and
    LB results equal the Python oracle's over the realized ServiceLB / EndpointDNAT flows and groups."""
    from antrea_amd import workload
    from tests import emu
    from tests.test_service import _oracle, _product
    base = workload.config1(seed=seed) if c1 else workload.config3(seed=seed, n_policies_per_dir=4, rules_per_policy=6)
    wl = workload.add_services(base, n_svc, eps, seed=seed, noep_frac=0.15, local_policy_frac=0.25)
    n = 300
    cols = workload.gen_packets(wl, n, seed=seed)
    c = _product(wl)
    lb = np.zeros(n, dtype=gpc.LB_DTYPE)
    got = emu.classify(c, cols, lb=lb)
    want, want_lb = _oracle(wl, c, cols, n)
    _cmp(got, want, cols)
    assert (lb == want_lb).all()
