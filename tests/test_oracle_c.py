"""The C oracle (OVS tuple-space-search restatement) agrees with the Python oracle."""
import copy

import numpy as np
import pytest

from antrea_amd import workload
from oracle import compiler as oc
from oracle import ovs_cls
from oracle.cls_c import CPipeline
from tests.util import load_golden, assign_tables

ACT = {"NONE": 0, "NO_MATCH": 1, "ALLOW": 2, "DROP": 3, "REJECT": 4, "ISOLATION_DROP": 5, "BYPASS": 6}


def test_c_oracle_appendix_a():
    import ipaddress
    batch = {c["name"]: c for c in load_golden("np_batch_install.json")["cases"]}
    for s in load_golden("appendix_a.json")["sets"]:
        pipe = CPipeline(batch[s["flows_from_case"]]["expected_flows"])
        pk = [tc["pkt"] for tc in s["packets"]]
        cols = {k: np.array([int(ipaddress.ip_address(p[k])) if k in ("src", "dst") else int(p.get(k, 0)) for p in pk])
                for k in ("src", "dst", "proto", "sport", "dport", "out_port", "tun_id")}
        got = pipe.classify(cols)
        for i, tc in enumerate(s["packets"]):
            for j, key in enumerate(("egress", "ingress")):
                a, conj, table, flags = tc[key]
                v = got[i, j]
                assert (v["action"], v["conj_id"], v["table"], v["flags"]) == (ACT[a], conj, table, flags), (tc, key)


@pytest.mark.parametrize("name,seed", [("C1", 1), ("C1", 2), ("C3s", 1), ("C3s", 2), ("C3s", 3)])
def test_c_vs_python_oracle(name, seed):
    wl = workload.config1(seed=seed) if name == "C1" else workload.config3(seed=seed, n_policies_per_dir=6,
                                                                              rules_per_policy=8)
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    flows = fnp.dump_flows()
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    n = 400
    cols = workload.gen_packets(wl, n, seed=seed)
    cols["len"] = np.full(n, 100, np.uint16)
    py = ovs_cls.Pipeline(flows, tiers)
    c = CPipeline(flows, tiers)
    got = c.classify(cols, threads=2, count=True)
    for i in range(n):
        e, g = py.classify({k: int(v[i]) for k, v in cols.items()})
        for j, v in enumerate((e, g)):
            assert tuple(got[i, j][["action", "conj_id", "table", "tier", "flags"]].item()) == v, (i, j)


@pytest.fixture(scope="module")
def full_c3():
    """Full-size C3 (100k rules). The C oracle consumes the product compiler's flow dump; that dump
    is itself pinned against the oracle compiler (tests/test_abi_compiler.py)."""
    from antrea_amd import gpc
    wl = workload.config3()
    clf = gpc.Classifier()
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    flows = clf.dump_flows()
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    return wl, clf, CPipeline(flows, tiers)


def test_emu_vs_c_oracle_full_c3(full_c3):
    from tests import emu
    wl, clf, pipe = full_c3
    emu.commit_host(clf)
    n = 4000
    cols = workload.gen_packets(wl, n, seed=77)
    want = pipe.classify(cols, threads=8)
    got = emu.classify(clf, cols)
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert len(bad) == 0, (len(bad), got[bad[0]], want[bad[0]])


def test_emu_vs_c_oracle_full_c2():
    """Full-size C2 (1k rules over AddressGroups of 50-1000 Pod IPs): the group clauses are point
    sets in the image's point hash and the driver entries probe them during the candidate scan;
    verdicts equal the C oracle's."""
    from antrea_amd import gpc
    from tests import emu
    wl = workload.config2()
    clf = gpc.Classifier()
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    pipe = CPipeline(clf.dump_flows(), tiers)
    emu.commit_host(clf)
    assert clf.image_stats()["bytes"]["hash"] > 1 << 20  # the group clauses did go to the point hash
    n = 20000
    cols = workload.gen_packets(wl, n, seed=78)
    want = pipe.classify(cols, threads=8)
    got = emu.classify(clf, cols)
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert len(bad) == 0, (len(bad), got[bad[0]], want[bad[0]])
    assert (got["action"] == ACT["ALLOW"]).sum() > n // 50
