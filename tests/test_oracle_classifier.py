"""Oracle classifier (OVS semantics) vs the hand-derived known answers of SURVEY Appendix A."""
import copy
import ipaddress

import pytest

from oracle import compiler as oc
from oracle import ovs_cls
from tests.util import assign_tables, load_golden

ACT = {"NONE": 0, "NO_MATCH": 1, "ALLOW": 2, "DROP": 3, "REJECT": 4, "ISOLATION_DROP": 5, "BYPASS": 6}
BATCH = {c["name"]: c for c in load_golden("np_batch_install.json")["cases"]}
APPX = load_golden("appendix_a.json")


def _pkt(d):
    p = dict(d)
    p["src"] = int(ipaddress.ip_address(p["src"]))
    p["dst"] = int(ipaddress.ip_address(p["dst"]))
    return p


@pytest.mark.parametrize("s", APPX["sets"], ids=[s["flows_from_case"] for s in APPX["sets"]])
def test_appendix_a_on_golden_flow_text(s):
    # classify against the reference's own golden flow strings (not our compiler's output)
    pipe = ovs_cls.Pipeline(BATCH[s["flows_from_case"]]["expected_flows"])
    for tc in s["packets"]:
        e, i = pipe.classify(_pkt(tc["pkt"]))
        want_e = (ACT[tc["egress"][0]], tc["egress"][1], tc["egress"][2], 0, tc["egress"][3])
        want_i = (ACT[tc["ingress"][0]], tc["ingress"][1], tc["ingress"][2], 0, tc["ingress"][3])
        assert (e, i) == (want_e, want_i), tc


@pytest.mark.parametrize("s", APPX["sets"], ids=[s["flows_from_case"] for s in APPX["sets"]])
def test_appendix_a_on_compiled_flows(s):
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(assign_tables(copy.deepcopy(BATCH[s["flows_from_case"]]["rules"])))
    pipe = ovs_cls.Pipeline(fnp.dump_flows())
    for tc in s["packets"]:
        e, i = pipe.classify(_pkt(tc["pkt"]))
        assert e[0] == ACT[tc["egress"][0]] and e[1] == tc["egress"][1]
        assert i[0] == ACT[tc["ingress"][0]] and i[1] == tc["ingress"][1]


def test_established_packets_bypass():
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(assign_tables(copy.deepcopy(BATCH["multiple K8s NetworkPolicy rules"]["rules"])))
    pipe = ovs_cls.Pipeline(fnp.dump_flows())
    p = _pkt({"src": "192.168.1.51", "dst": "10.0.0.1", "proto": 17, "sport": 1, "dport": 53,
              "ct_state": ovs_cls.CT_EST | ovs_cls.CT_TRK})
    e, i = pipe.classify(p)
    assert e[0] == ovs_cls.ACT_BYPASS and i[0] == ovs_cls.ACT_BYPASS


def test_metric_counters_roundtrip():
    """Counters land on the Metric-table flows and parse back through NetworkPolicyMetrics."""
    fnp = oc.FeatureNetworkPolicy()
    fnp.batch_install_policy_rule_flows(assign_tables(copy.deepcopy(BATCH["multiple Antrea NetworkPolicy rules"]["rules"])))
    pipe = ovs_cls.Pipeline(fnp.dump_flows())
    for tc in APPX["sets"][0]["packets"]:
        p = _pkt(tc["pkt"])
        p["len"] = 100
        pipe.classify(p)
    d = pipe.metric_dumps()
    m = oc.network_policy_metrics(d["EgressMetric"], d["IngressMetric"])
    assert m[10] == (2, 200, 2)
    assert m[12] == (2, 200, 2)
    assert m[11] == (1, 100, 1)
    assert m[14] == (1, 100, 1)
