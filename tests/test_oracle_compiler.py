"""Oracle compiler vs the reference's golden flow strings (network_policy_test.go)."""
import copy

import pytest

from oracle import compiler as oc
from tests.util import assign_tables, load_golden, normalize_flows

GOLD = load_golden("np_batch_install.json")


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_batch_install_golden(case):
    rules = assign_tables(copy.deepcopy(case["rules"]))
    fnp = oc.FeatureNetworkPolicy()
    flows = fnp.batch_install_policy_rule_flows(rules)
    got = normalize_flows([oc.flow_to_string(f) for f in flows])
    want = normalize_flows(case["expected_flows"])
    assert got == want, "\nmissing: %s\nextra: %s" % (sorted(want - got), sorted(got - want))


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_incremental_install_equals_batch(case):
    """InstallPolicyRuleFlows one by one realizes the same flow table as BatchInstall."""
    rules = assign_tables(copy.deepcopy(case["rules"]))
    a = oc.FeatureNetworkPolicy()
    a.batch_install_policy_rule_flows(rules)
    b = oc.FeatureNetworkPolicy()
    for r in rules:
        b.install_policy_rule_flows(r)
    assert normalize_flows(a.dump_flows()) == normalize_flows(b.dump_flows())
    assert normalize_flows(b.dump_flows()) == normalize_flows(case["expected_flows"])


def test_bitwise_match_known_ranges():
    # port_range.go:45-132 (go-openvswitch portrange): 1000-1007 is one aligned block (used by
    # network_policy_test.go:251-283), 5-8 needs three blocks.
    assert oc.bitwise_match(1000, 1007) == [(1000, 0xFFF8)]
    assert oc.bitwise_match(5, 8) == [(5, 0xFFFF), (6, 0xFFFE), (8, 0xFFFF)]
    assert oc.bitwise_match(80, 80) == [(80, 0xFFFF)]


@pytest.mark.parametrize("seed", range(20))
def test_bitwise_match_exact_cover(seed):
    import random
    rng = random.Random(seed)
    for _ in range(50):
        a = rng.randint(1, 65535)
        b = rng.randint(a, min(65535, a + rng.choice([1, 7, 100, 5000, 65535])))
        blocks = oc.bitwise_match(a, b)
        covered = set()
        for v, m in blocks:
            size = (~m & 0xFFFF) + 1
            assert v & ~m & 0xFFFF == 0
            rng_ = set(range(v, v + size))
            assert not (covered & rng_)
            covered |= rng_
        assert covered == set(range(a, b + 1))


def _k8s_rule(fid, frm, to=None, svc=None):
    r = {"direction": "Out", "from": frm, "flow_id": fid, "table": "EgressRule",
         "policy_type": "K8sNetworkPolicy", "policy_namespace": "ns1", "policy_name": "np1"}
    if to is not None:
        r["to"] = to
    if svc is not None:
        r["service"] = svc
    return r


def _changes(fnp, rule):
    conj = fnp.calculate_action_flows(rule)
    chs = []
    for clause, m in fnp._rule_matches(conj, rule):
        ch = fnp._add_conjunctive_match_flow(clause, m, False, False)
        if ch is not None:
            chs.append(ch)
    return conj, chs


def _count(chs, which, typ=None, with_flow=True):
    n = 0
    for ch in chs:
        fc = ch[which]
        if fc is None:
            continue
        if with_flow and fc[1] is None:
            continue
        if typ is None or fc[0] == typ:
            n += 1
    return n


def test_install_change_counts():
    """TestInstallPolicyRuleFlows (network_policy_test.go:165-310) change counts."""
    fnp = oc.FeatureNetworkPolicy()
    r1 = _k8s_rule(101, ["192.168.1.30", "192.168.1.50"])
    conj1, ch = _changes(fnp, r1)
    assert conj1.to_clause is None and conj1.service_clause is None
    assert len(ch) == 2
    assert _count(ch, "drop") == 2
    assert _count(ch, "match_flow") == 0
    assert sum(1 for c in ch if c["match_flow"] == ("insertion", None)) == 2
    fnp._apply_changes(ch)

    r2 = _k8s_rule(102, ["192.168.1.40", "192.168.1.50"], to=["0.0.0.0/0"])
    conj2, ch = _changes(fnp, r2)
    assert _count(ch, "drop") == 1
    assert _count(ch, "match_flow") == 3
    assert _count(ch, "match_flow", "insertion") == 3
    fnp._apply_changes(ch)
    fnp.policy_cache[conj2.id] = conj2

    r3 = _k8s_rule(103, ["192.168.1.40", "192.168.1.60"], to=["192.168.2.0/24"],
                   svc=[{"protocol": "TCP", "port": 8080}, {"protocol": "TCP", "port": 1000, "end_port": 1007},
                        {"protocol": "ICMP", "icmp_type": 8, "icmp_code": 0}])
    conj3, ch = _changes(fnp, r3)
    assert _count(ch, "drop", "insertion") == 1
    assert _count(ch, "match_flow") == 6
    assert _count(ch, "match_flow", "insertion") == 5
    assert _count(ch, "match_flow", "modification") == 1
    fnp._apply_changes(ch)
    fnp.policy_cache[conj3.id] = conj3

    # delete rule 1 (DENY-ALL): one drop flow deleted (.30), two deny-all ops
    chs = []
    for cl in conj1.clauses():
        for key in list(cl.matches):
            c = fnp._delete_conjunctive_match_flow(cl, key)
            if c:
                chs.append(c)
    assert _count(chs, "drop", "deletion") == 1
    assert sum(1 for c in chs if c["match_flow"] == ("deletion", None)) == 2
    fnp._apply_changes(chs)

    # delete rule 2: drop .50 goes; .40 stays (used by rule 3); flows: 2 deletions + 1 modification
    chs = []
    for cl in conj2.clauses():
        for key in list(cl.matches):
            c = fnp._delete_conjunctive_match_flow(cl, key)
            if c:
                chs.append(c)
    assert _count(chs, "drop", "deletion") == 1
    assert _count(chs, "match_flow") == 3
    assert _count(chs, "match_flow", "deletion") == 2
    assert _count(chs, "match_flow", "modification") == 1


def test_conj_match_flow_context_key_conflict():
    """TestConjMatchFlowContextKeyConflict (network_policy_test.go:627-669): IP and IP/32 share one
    context."""
    fnp = oc.FeatureNetworkPolicy()
    c1 = oc.Conjunction(11)
    cl1 = oc.Clause(oc.ConjAction(11, 1, 3), "EgressRule", "EgressDefaultRule")
    c2 = oc.Conjunction(12)
    cl2 = oc.Clause(oc.ConjAction(12, 1, 3), "EgressRule", "EgressDefaultRule")
    for cl, addr in ((cl1, "192.168.2.30"), (cl2, "192.168.2.30/32")):
        a = oc.parse_address(addr)
        m = oc.ConjunctiveMatch("EgressRule", None, [(oc.address_match_key(a, False), oc.address_match_value(a))])
        fnp._apply_changes([fnp._add_conjunctive_match_flow(cl, m, False, False)])
    assert len(fnp.global_cache) == 1
    ctx = next(iter(fnp.global_cache.values()))
    assert set(ctx.actions) == {11, 12}


def test_metric_parse_golden():
    """TestParseMetricFlow / TestNetworkPolicyMetrics (network_policy_test.go:1061-1195)."""
    g = load_golden("np_metrics.json")
    for tc in g["parse"]:
        rid, m = oc.parse_metric_flow(oc.parse_flow_to_map(tc["flow"]))
        assert rid == tc["rule"] and list(m) == tc["metric"]
    for tc in g["metrics"]:
        got = oc.network_policy_metrics(tc["egress"], tc["ingress"])
        want = {int(k): tuple(v) for k, v in tc["want"].items()}
        assert got == want
