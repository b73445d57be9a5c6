"""GPU tier at the BASELINE sizes: the HIP path (gpc_classify through the C-ABI) against the C
oracle's verdicts and per-rule metrics, packet for packet.

The oracle side is the committed fixture tests/golden/parity_<config>.npz, generated on the CPU by
tests/golden/make_parity_fixtures.py: the ORACLE compiler's flows for the full workload (C2: 1k
rules over AddressGroups of up to 1000 Pod IPs; C3: 100k rules, 1.67M flows; C4: C3 + 10k
Services), classified by the C restatement of the OVS classifier (oracle/ovs_cls.c) with counters.
Each test regenerates the same seeded inputs and first checks their SHA-256 against the fixture's,
so the device and the oracle always classify identical packets under identical rules."""
import copy
import os

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import parity
from tests.golden import make_parity_fixtures as fx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


def _classifier(wl, ipv6=False, rules=None, group=0):
    c = gpc.Classifier(ipv4=not ipv6, ipv6=ipv6, group_packets=group)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(rules if rules is not None else wl.rules))
    if getattr(wl, "services", None):
        workload.install_services(c, wl)
    c.commit()
    return c


def _inputs(config):
    f = fx.load(config)
    wl, cols = fx.packets(config)
    assert fx.cols_digest(cols) == str(f["cols_sha256"]), "packet generator drifted from the fixture"
    assert fx.rules_digest(wl) == str(f["rules_sha256"]), "rule generator drifted from the fixture"
    return f, wl, cols


def _nonzero(m):
    return {int(k): tuple(int(x) for x in v) for k, v in m.items() if any(v)}


@pytest.mark.parametrize("group", [-1, 1], ids=["plain", "grouped"])
@pytest.mark.parametrize("config", ["C1", "C2", "C3", "C4", "C3x"])
def test_device_vs_oracle_fullscale(config, group):
    """Verdicts (conj id, action, table, tier, flags) and NetworkPolicyMetrics of 100k packets at
    full scale equal the C oracle's exactly (C4: every packet, the Service stage's LB results too,
    against the C oracle's AntreaProxy stage; C3x: C3 with every optional column set -- conntrack states, pre-NAT
    addresses, IngressSecurityClassifier destinations and hairpin mark, in_port, tun_id, reg7),
    with the packet grouping pre-pass off and on (the bench's 64M-packet batches are grouped)."""
    f, wl, cols = _inputs(config)
    c = _classifier(wl, group=group)
    if "lb" in f:  # C4: the LB result words of every packet against the oracle's AntreaProxy stage
        got, lb = c.classify_host(cols, count=True, lb=True)
        bad = np.nonzero((lb.view(np.uint32).reshape(-1, 4) != f["lb"]).any(axis=1))[0]
        assert len(bad) == 0, (len(bad), bad[:5])
    else:
        got = c.classify_host(cols, count=True)
    res = parity.compare(got, f["verdicts"])
    assert res["mismatches"] == 0, res
    assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"])
    acts = set(int(a) for a in np.unique(got["action"]))
    # NO_MATCH, ALLOW and a deny (ACNP DROP; K8s NP isolation drop for C1) all exercised
    assert {1, 2} <= acts and (3 in acts or 5 in acts), acts


def test_device_vs_oracle_c2g():
    """BASELINE configs[1] as worded: 1k ACNP rules whose From clauses are
    AddressGroups of 10k Pod IPs each (16 groups over the 10.0.0.0/16 Pods, 10M conjunctive match
    flows). Verdicts and metrics of 100k packets equal the C oracle's (fixture built from the
    oracle compiler's 10M flows, tests/golden/parity_C2g.npz)."""
    f, wl, cols = _inputs("C2g")
    c = _classifier(wl)
    assert c.image_stats()["n_flows"] > 10_000_000
    got = c.classify_host(cols, count=True)
    res = parity.compare(got, f["verdicts"])
    assert res["mismatches"] == 0, res
    assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"])
    acts = set(int(a) for a in np.unique(got["action"]))
    assert {1, 2, 3} <= acts, acts


@pytest.mark.parametrize("config", ["C2", "C3"])
def test_device_vs_oracle_fullscale_plain_driver(config, monkeypatch):
    """The same parity with the composite driver index turned off (GPC_COMPOSITE=0, read at image
    build): tables then keep the plain per-clause driver indexes, the kernel's other lookup path."""
    monkeypatch.setenv("GPC_COMPOSITE", "0")
    f, wl, cols = _inputs(config)
    c = _classifier(wl, group=1)
    got = c.classify_host(cols, count=True)
    res = parity.compare(got, f["verdicts"])
    assert res["mismatches"] == 0, res
    assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"])


@pytest.mark.parametrize("group", [-1, 1], ids=["plain", "grouped"])
def test_device_ipv6_vs_oracle_fullscale_c3(group):
    """gpc_classify6 on full C3 embedded in fd00:10::/96 (IPv6 image, device LPM) equals the C
    oracle's IPv4 verdicts of the same packets (the embedding preserves every match), with the
    grouping pre-pass off and on (IPv6 batches are grouped over their code columns: the top byte
    of the source address's code)."""
    f, wl, cols = _inputs("C3")
    c = _classifier(wl, ipv6=True, rules=workload.to_ipv6(wl).rules, group=group)
    got = c.classify6_host(workload.packets_to_v6(cols), count=True)
    res = parity.compare(got, f["verdicts"])
    assert res["mismatches"] == 0, res
    assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"])


def test_device_ipv6_multi48_vs_oracle_fullscale_c3():
    """Full C3 embedded over four /48s (workload "multi48": the top 2 IPv4 bits pick the /48) -- the
    device LPM's region tables then have one table per tag (rule sets over several
    /48s) -- equals the C oracle's IPv4 verdicts of the same packets."""
    f, wl, cols = _inputs("C3")
    c = _classifier(wl, ipv6=True, rules=workload.to_ipv6(wl, embed="multi48").rules)
    got = c.classify6_host(workload.packets_to_v6(cols, embed="multi48"), count=True)
    res = parity.compare(got, f["verdicts"])
    assert res["mismatches"] == 0, res
    assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"])


@pytest.mark.parametrize("dual", [False, True])
def test_device_ipv6_vs_python_oracle_c1(dual):
    """gpc_classify6 directly against the Python oracle over the oracle compiler's IPv6 flows
    (ipv6_src / ipv6_dst / tcp6 ...), C1 and C1 dual-stack."""
    from tests.test_ipv6 import _oracle6
    wl = workload.config1(seed=4)
    w6 = workload.to_ipv6(wl, dual=dual)
    n = 2000
    cols6 = workload.packets_to_v6(workload.gen_packets(wl, n, seed=4))
    want = _oracle6(w6.rules, cols6, n)
    c = _classifier(w6, ipv6=True)
    got = c.classify6_host(cols6)
    res = parity.compare(got, want)
    assert res["mismatches"] == 0, res


@pytest.mark.parametrize("group", [-1, 1], ids=["plain", "grouped"])
def test_device_vs_oracle_after_churn_c3(group):
    """Config 5's update path at full scale against the oracle: C3, then the seeded op log of
    tests/golden/make_churn_fixture.py (2125 AddPolicyRuleAddress, 869 DeletePolicyRuleAddress incl.
    original addresses, 200 UninstallPolicyRuleFlows, 99 reinstalls, 30 ReassignFlowPriorities)
    published as delta epochs every 100 ops (journal + tombstones; the background compactor may
    hand over meanwhile): verdicts and NetworkPolicyMetrics of 100k packets equal the C oracle's
    over the oracle compiler's replay of the same log -- then again after gpc_compact."""
    from tests.golden import make_churn_fixture as cf
    f = cf.load()
    wl, log, cols = cf.inputs()
    assert fx.cols_digest(cols) == str(f["cols_sha256"]) and fx.rules_digest(wl) == str(f["rules_sha256"])
    assert cf.log_digest(log) == str(f["log_sha256"]), "op log generator drifted from the fixture"
    c = _classifier(wl, group=group)
    cf.apply(c, log, on_commit=c.commit)
    assert c.image_stats()["n_delta_builds"] > 0
    for phase in ("delta", "compacted"):
        if phase == "compacted":
            c.compact()
            c.reset_counters()
        got = c.classify_host(cols, count=True)
        res = parity.compare(got, f["verdicts"])
        assert res["mismatches"] == 0, (phase, res)
        assert _nonzero(c.network_policy_metrics()) == _nonzero(f["metrics"]), phase
