"""The rest of the openflow.Client NetworkPolicy surface, pinned by the reference's own tests:

* initFlows (Initialize NP part)           network_policy_test.go:1363-1410
* NewDNSPacketInConjunction                network_policy_test.go:1454-1560 (+ Add/Delete address)
* GetNetworkPolicyFlowKeys counts          network_policy_test.go:243-308 (the public-API equivalent)
* GetPolicyInfoFromConjunction             network_policy_test.go:1288-1361

Each is checked on the oracle compiler and on the product library (C-ABI), which must agree.
CPU tier; the classification consequences (DNS interception verdict, IngressSecurityClassifier
bypass) are checked against the oracle through the host emulation here and on the device in
tests/test_gpu_boundary.py."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import compiler as oc
from oracle import ovs_cls
from tests import emu
from tests.test_emu_parity import _cmp
from tests.util import load_golden, normalize_flows

GOLD = load_golden("np_init_dns.json")


@pytest.mark.parametrize("case", GOLD["init_flows"], ids=lambda c: c["name"])
def test_init_flows_golden(case):
    want = normalize_flows(case["expected_flows"])
    fnp = oc.FeatureNetworkPolicy(ovs_meters=case["ovs_meters"], k8s_node=case["k8s_node"])
    fnp.initialize()
    assert normalize_flows(fnp.dump_flows()) == want
    c = gpc.Classifier(ovs_meters=case["ovs_meters"], k8s_node=case["k8s_node"])
    c.initialize()
    assert normalize_flows(c.dump_flows()) == want


@pytest.mark.parametrize("case", GOLD["dns_conjunction"], ids=lambda c: c["name"])
def test_dns_conjunction_golden(case):
    want = normalize_flows(case["expected_flows"])
    fnp = oc.FeatureNetworkPolicy(ipv4=case["ipv4"], ipv6=case["ipv6"], ovs_meters=case["ovs_meters"])
    fnp.new_dns_packet_in_conjunction(case["conj_id"])
    assert normalize_flows(fnp.dump_flows()) == want
    c = gpc.Classifier(ipv4=case["ipv4"], ipv6=case["ipv6"], ovs_meters=case["ovs_meters"])
    c.new_dns_packet_in_conjunction(case["conj_id"])
    c.new_dns_packet_in_conjunction(case["conj_id"])  # a second call is a no-op (network_policy.go:698-702)
    assert normalize_flows(c.dump_flows()) == want


def _dns_pair(addrs_add, addrs_del=()):
    fnp = oc.FeatureNetworkPolicy(ipv4=True, ipv6=True)
    fnp.initialize()
    c = gpc.Classifier(ipv4=True, ipv6=True)
    c.initialize()
    for side in (fnp, c):
        side.new_dns_packet_in_conjunction(7)
        side.add_address_to_dns_conjunction(7, list(addrs_add))
        if addrs_del:
            side.delete_address_from_dns_conjunction(7, list(addrs_del))
    return fnp, c


def test_dns_conjunction_addresses():
    """AddAddressToDNSConjunction / DeleteAddressFromDNSConjunction = Add/DeletePolicyRuleAddress
    of the to clause (2/2) at priority 64991 (network_policy.go:781-789)."""
    fnp, c = _dns_pair(["10.10.0.5", "10.10.0.6", "fd00::5"], ["10.10.0.6"])
    got = normalize_flows(c.dump_flows())
    assert got == normalize_flows(fnp.dump_flows())
    assert any("priority=64991,ip,nw_dst=10.10.0.5 actions=conjunction(7,2/2)" in f for f in got)
    assert any("priority=64991,ipv6,ipv6_dst=fd00::5 actions=conjunction(7,2/2)" in f for f in got)
    assert not any("10.10.0.6" in f for f in got)
    fnp.delete_address_from_dns_conjunction(7, ["10.10.0.5", "fd00::5"])
    c.delete_address_from_dns_conjunction(7, ["10.10.0.5", "fd00::5"])
    assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows())
    with pytest.raises(gpc.GpcError) as e:
        c.add_address_to_dns_conjunction(8, ["10.10.0.7"])  # not created: ConjunctionNotFound
    assert e.value.code == gpc.GPC_ENOTFOUND


def _dns_cols(n, rng, dns_ips):
    cols = {"src": rng.integers(0, 1 << 32, n).astype(np.uint32),
            "dst": np.where(rng.random(n) < 0.6, rng.choice(dns_ips, n), rng.integers(0, 1 << 32, n)).astype(np.uint32),
            "sport": np.where(rng.random(n) < 0.7, 53, rng.integers(1, 65536, n)).astype(np.uint16),
            "dport": rng.integers(1024, 65536, n).astype(np.uint16),
            "proto": rng.choice([6, 17, 1], n).astype(np.uint8),
            "out_port": rng.integers(3, 10, n).astype(np.uint32),
            "ct_state": rng.choice([0x21, 0x28, 0x2a, 0x22], n).astype(np.uint8)}
    return cols


def test_dns_interception_verdicts_emu_vs_oracle():
    """Solicited DNS responses (ct_state=+rpl+trk, sport 53) to the DNS conjunction's Pods: BYPASS
    to IngressMetric with PACKETIN, exactly as the oracle walks the dnsPacketInFlow; everything else
    continues through the policy tables (C1 rules installed alongside)."""
    wl = workload.config1(seed=12)
    ips = [int(x) for x in wl.local_ips[:5]]
    addrs = ["%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255) for v in ips]
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    fnp.new_dns_packet_in_conjunction(9999)
    fnp.add_address_to_dns_conjunction(9999, addrs)
    c = gpc.Classifier()
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    c.new_dns_packet_in_conjunction(9999)
    c.add_address_to_dns_conjunction(9999, addrs)
    emu.commit_host(c)
    assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows())
    rng = np.random.default_rng(12)
    n = 600
    cols = _dns_cols(n, rng, np.array(ips, np.uint32))
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), {r["flow_id"]: 0 for r in wl.rules})
    want = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for i in range(n):
        e, g = pipe.classify({k: int(v[i]) for k, v in cols.items()})
        for j, v in enumerate((e, g)):
            want[i, j] = (v[1], v[0], v[2], v[3], v[4])
    got = emu.classify(c, cols)
    _cmp(got, want, cols)
    pin = (got[:, 1]["flags"] & 4) != 0
    assert pin.sum() > 20 and (got[pin, 1]["action"] == 6).all()


def test_ingress_classifier_bypass_emu_vs_oracle():
    """IngressSecurityClassifier (pipeline.go:2144-2182), data-driven from the installed flows:
    packets to the gateway / tunnel / uplink go to IngressMetric and hairpin connections
    (ct_mark=0x40/0x40) to ConntrackCommit, both BYPASS; both at once is an equal-priority overlap
    of different actions (TIE). On an ExternalNode (no classifier flows) they take the tables."""
    wl = workload.config1(seed=13)
    n = 800
    cols = workload.gen_packets(wl, n, seed=13)
    rng = np.random.default_rng(13)
    cols["dest"] = rng.choice([0, 0, 1, 2, 3], n).astype(np.uint8)
    cols["ct_mark"] = np.where(rng.random(n) < 0.25, 0x40, rng.choice([0, 0x10, 0x20], n)).astype(np.uint8)
    for k8s in (True, False):
        fnp = oc.FeatureNetworkPolicy(k8s_node=k8s)
        fnp.initialize()
        fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        pipe = ovs_cls.Pipeline(fnp.dump_flows(), {})
        want = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
        for i in range(n):
            e, g = pipe.classify({k: int(v[i]) for k, v in cols.items()})
            for j, v in enumerate((e, g)):
                want[i, j] = (v[1], v[0], v[2], v[3], v[4])
        c = gpc.Classifier(k8s_node=k8s)
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        emu.commit_host(c)
        got = emu.classify(c, cols)
        _cmp(got, want, cols)
        byp = got[:, 1]["action"] == 6
        if k8s:
            assert byp.sum() > n // 4 and ((got[byp, 1]["flags"] & 2) != 0).any()
        else:
            assert not byp.any()


def _rule(fid, frm, to=None, svc=None, name="np1", prio=None, table="EgressRule", direction="Out", log_label=""):
    r = {"direction": direction, "table": table, "flow_id": fid, "policy_type": "K8sNetworkPolicy",
         "policy_namespace": "ns1", "policy_name": name, "policy_uid": "id1", "from": frm, "to": to,
         "service": svc, "name": str(fid), "log_label": log_label}
    if prio is not None:
        r["priority"] = prio
    return r


def test_network_policy_flow_keys():
    """TestInstallPolicyRuleFlows' GetNetworkPolicyFlowKeys counts (network_policy_test.go:243-308)
    through the public API: a DNS conjunction (no NetworkPolicyReference, ignored), rule 101 (a
    DENY-ALL From-only rule, here of another policy so np1's counts match), rule 102 -> 6 keys,
    rule 103 with TCP 8080 / TCP 1000-1007 / ICMP 8/0 -> 15, and after uninstalling 102 -> 9."""
    r1 = _rule(101, ["192.168.1.30", "192.168.1.50"], name="np0")
    r2 = _rule(102, ["192.168.1.40", "192.168.1.50"], to=["0.0.0.0/0"])
    r3 = _rule(103, ["192.168.1.40", "192.168.1.60"], to=["192.168.2.0/24"],
               svc=[{"protocol": "TCP", "port": 8080}, {"protocol": "TCP", "port": 1000, "end_port": 1007},
                    {"protocol": "ICMP", "icmp_type": 8, "icmp_code": 0}])
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.new_dns_packet_in_conjunction(1)
        side.install_policy_rule_flows(copy.deepcopy(r1))
    keys = lambda s: s.get_network_policy_flow_keys("np1", "ns1", "K8sNetworkPolicy")
    assert len(keys(fnp)) == len(keys(c)) == 0
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r2))
    assert len(keys(fnp)) == len(keys(c)) == 6
    assert sorted(keys(fnp)) == sorted(keys(c))
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r3))
    assert len(keys(fnp)) == len(keys(c)) == 15
    assert "table=EgressRule,conj_id=103,ip" in keys(c)
    assert "table=EgressRule,tcp,tp_dst=0x3e8/0xfff8" in keys(c)
    for side in (fnp, c):
        side.uninstall_policy_rule_flows(102)
    assert sorted(keys(fnp)) == sorted(keys(c)) and len(keys(c)) == 9
    assert c.get_network_policy_flow_keys("np0", "ns1", "K8sNetworkPolicy") != []
    assert c.get_network_policy_flow_keys("np1", "ns1", "AntreaNetworkPolicy") == []


def test_get_policy_info_from_conjunction():
    """TestClient_GetPolicyInfoFromConjunction (network_policy_test.go:1288-1361): not found;
    found but no action flows (empty priorities); found with priority "100", the rule name and the
    log label. Conjunction 102's only action flow has priority 100."""
    r101 = _rule(101, ["1.1.1.10"])  # one clause: DENY-ALL, no action flows
    r102 = _rule(102, ["1.1.1.10"], to=["1.1.1.0/24"], prio=100, log_label="test-log-label")
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r101))
        side.install_policy_rule_flows(copy.deepcopy(r102))
        side.new_dns_packet_in_conjunction(5)  # no NetworkPolicyReference
    for side in (fnp, c):
        assert side.get_policy_info_from_conjunction(100)[0] is False
        assert side.get_policy_info_from_conjunction(101)[0] is False
        assert side.get_policy_info_from_conjunction(5)[0] is False
        ok, ref, prio, name, label = side.get_policy_info_from_conjunction(102)
        assert ok and prio == "100" and name == "102" and label == "test-log-label"
        assert "%s:%s/%s" % (ref[0], ref[1], ref[2]) == "K8sNetworkPolicy:ns1/np1"  # NetworkPolicyReference.ToString


def test_network_policy_flow_keys_dual_stack():
    """TestInstallPolicyRuleFlowsInDualStackCluster (network_policy_test.go:671-810) through the
    public API: with IPv4 and IPv6 enabled, K8s rule 102 (From two IPv4 + one IPv6 address, To
    0.0.0.0/0) realizes 2 conj_id flows (ip, ipv6) + 4 conjunctive match flows + 3 drop flows = 9
    keys, and rule 103 (TCP 8080 / 8081, matched as tcp and tcp6) brings np1 to 20. Rule 101 is the
    DENY-ALL From-only rule, here of another policy (the reference applies its flows without
    registering it). Product and oracle compilers give identical dumps and keys."""
    r1 = _rule(101, ["192.168.1.30", "192.168.1.50", "fd12:ab:34:a001::4"], name="np0")
    r2 = _rule(102, ["192.168.1.40", "192.168.1.50", "fd12:ab:34:a001::5"], to=["0.0.0.0/0"])
    r3 = _rule(103, ["192.168.1.40", "192.168.1.60"], to=["192.168.2.0/24"],
               svc=[{"protocol": "TCP", "port": 8080}, {"protocol": "TCP", "port": 8081}])
    fnp, c = oc.FeatureNetworkPolicy(ipv4=True, ipv6=True), gpc.Classifier(ipv4=True, ipv6=True)
    keys = lambda s: sorted(s.get_network_policy_flow_keys("np1", "ns1", "K8sNetworkPolicy"))
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r1))
    # DENY-ALL: one drop flow per From address in EgressDefaultRule, no conjunction
    drops = [f for f in c.dump_flows() if "table=EgressDefaultRule" in f]
    assert len(drops) == 3 and any("ipv6_src=fd12:ab:34:a001::4" in f for f in drops)
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r2))
    assert len(keys(c)) == 9 and keys(c) == keys(fnp)
    assert "table=EgressRule,conj_id=102,ipv6" in keys(c)
    for side in (fnp, c):
        side.install_policy_rule_flows(copy.deepcopy(r3))
    assert len(keys(c)) == 20 and keys(c) == keys(fnp)
    assert "table=EgressRule,tcp6,tp_dst=0x1f90" in keys(c) or "table=EgressRule,tcp6,tp_dst=8080" in keys(c)
    assert normalize_flows(c.dump_flows()) == normalize_flows(fnp.dump_flows())


def test_get_match_flow_updates_reassign():
    """TestGetMatchFlowUpdates (network_policy_test.go:1197-1273): ANNP rules 10 / 11 at priority 100
    share the nw_src=192.168.1.40 conjunctive match flow, rule 12 at 200 has its own; after
    ReassignFlowPriorities {100: 101, 200: 202} the shared flow carries both conjunctions at 101 and
    rule 12's at 202 -- product and oracle dumps identical, no flow left at the old priorities."""
    def annp(fid, frm, ports, prio, action, svc=None):
        r = _rule(fid, frm, to=[{"ofport": p} for p in ports], svc=svc, name="np%d" % fid, prio=prio,
                  table="AntreaPolicyEgressRule")
        r.update(policy_type="AntreaNetworkPolicy", action=action)
        return r
    tcp8080 = [{"protocol": "TCP", "port": 8080}]
    rules = [annp(10, ["192.168.1.40", "192.168.1.50"], [1, 2], 100, "Allow"),
             annp(11, ["192.168.1.40", "192.168.1.51"], [1, 3], 100, "Drop", tcp8080),
             annp(12, ["192.168.1.40"], [1], 200, "Drop", tcp8080)]
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.initialize()
        side.batch_install_policy_rule_flows(copy.deepcopy(rules))
    before = [f for f in c.dump_flows() if "nw_src=192.168.1.40" in f]
    assert any("priority=100" in f and "conjunction(10,1/2)" in f and "conjunction(11,1/3)" in f for f in before)
    assert any("priority=200" in f and "conjunction(12,1/3)" in f for f in before)
    for side in (fnp, c):
        side.reassign_flow_priorities({100: 101, 200: 202}, "AntreaPolicyEgressRule")
    got = c.dump_flows()
    assert normalize_flows(got) == normalize_flows(fnp.dump_flows())
    ap = [f for f in got if "table=AntreaPolicyEgressRule" in f]
    assert not any("priority=100," in f or "priority=200," in f for f in ap)
    assert any("priority=101" in f and "nw_src=192.168.1.40" in f and "conjunction(10,1/2)" in f for f in ap)
    assert any("priority=202" in f and "conj_id=12" in f for f in ap)


def test_group_key_config_validated():
    """gpc_config.group_key: AUTO / ADDR / SCAN are accepted, anything else is -GPC_EINVAL at
    gpc_create (no device work)."""
    for k in (gpc.GROUP_KEY_AUTO, gpc.GROUP_KEY_ADDR, gpc.GROUP_KEY_SCAN):
        gpc.Classifier(group_key=k)
    for k in (-1, 3):
        with pytest.raises(gpc.GpcError) as e:
            gpc.Classifier(group_key=k)
        assert e.value.code == gpc.GPC_EINVAL
