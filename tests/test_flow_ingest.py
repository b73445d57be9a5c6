"""Flow-text ingest: gpc_load_flows parses ovs-ofctl flow text into the realized
table; the image built from it must classify exactly like the compiled rules it came from, and
like the oracle on the reference's own golden flow strings (network_policy_test.go:349-364,
447-475) with the SURVEY Appendix A answers."""
import copy
import ipaddress

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import ovs_cls
from tests import emu
from tests.test_emu_parity import _cmp
from tests.util import load_golden, normalize_flows

ACT = {"NONE": 0, "NO_MATCH": 1, "ALLOW": 2, "DROP": 3, "REJECT": 4, "ISOLATION_DROP": 5, "BYPASS": 6}
BATCH = {c["name"]: c for c in load_golden("np_batch_install.json")["cases"]}
APPX = load_golden("appendix_a.json")


def _compiled(wl):
    c = gpc.Classifier()
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    emu.commit_host(c)
    return c


@pytest.mark.parametrize("name", ["C1", "C3s"])
def test_roundtrip_dump_load(name):
    wl = workload.config1(seed=41) if name == "C1" else workload.config3(seed=41, n_policies_per_dir=10,
                                                                            rules_per_policy=20)
    src = _compiled(wl)
    dump = src.dump_flows()
    dst = gpc.Classifier()
    loaded, skipped = dst.load_flows(dump)
    assert loaded == len(dump) and skipped == 0
    assert normalize_flows(dst.dump_flows()) == normalize_flows(dump)
    emu.commit_host(dst)
    cols = workload.gen_packets(wl, 20000, seed=41)
    a, b = emu.classify(src, cols), emu.classify(dst, cols)
    # loaded flows carry no tier (a PolicyRule attribute, not a flow field): compare without it
    a["tier"] = 0
    b["tier"] = 0
    _cmp(b, a, cols)
    st = dst.image_stats()
    assert st["n_full_builds"] == 1 and st["n_flows"] == len(dump)


def _pk(d):
    return {k: (int(ipaddress.ip_address(v)) if k in ("src", "dst") else int(v)) for k, v in d.items()}


@pytest.mark.parametrize("s", APPX["sets"], ids=[s["flows_from_case"] for s in APPX["sets"]])
def test_appendix_a_on_loaded_golden_flows(s):
    """The reference's golden flow strings, loaded as text, give the Appendix A verdicts."""
    flows = BATCH[s["flows_from_case"]]["expected_flows"]
    c = gpc.Classifier()
    n, _ = c.load_flows(flows)
    assert n == len(flows)
    emu.commit_host(c)
    pk = [_pk(tc["pkt"]) for tc in s["packets"]]
    cols = {k: np.array([p.get(k, 0) for p in pk], dtype=np.int64)
            for k in ("src", "dst", "proto", "sport", "dport", "out_port", "tun_id")}
    got = emu.classify(c, cols)
    pipe = ovs_cls.Pipeline(flows)
    for i, tc in enumerate(s["packets"]):
        want = pipe.classify(pk[i])
        for j, key in enumerate(("egress", "ingress")):
            a, conj, table, flags = tc[key]
            v = got[i, j]
            assert (v["action"], v["conj_id"], v["table"], v["flags"]) == (ACT[a], conj, table, flags), (tc, key, v)
            assert (v["action"], v["conj_id"], v["table"], v["flags"]) == (want[j][0], want[j][1], want[j][2],
                                                                          want[j][4])


def test_dump_flows_format_and_foreign_tables():
    """`ovs-ofctl dump-flows --names` lines (stats fields, resubmit, other pipeline tables)."""
    flows = BATCH["multiple Antrea NetworkPolicy rules"]["expected_flows"]
    dumped = []
    for f in flows:
        head, rest = f.split("table=", 1)
        cookie = head.strip().rstrip(",")
        dumped.append(" %s duration=12.5s, table=%s" % (cookie + "," if cookie else "", rest.replace(
            " priority=", " n_packets=7, n_bytes=700, idle_age=3, priority=", 1)))
    dumped += ["NXST_FLOW reply (xid=0x4):",
               " cookie=0x1000000000000, duration=9.1s, table=Classifier, n_packets=0, n_bytes=0, priority=200,"
               "in_port=2 actions=set_field:0x2/0xf->reg0,goto_table:SpoofGuard",
               " cookie=0x1000000000000, table=Output, priority=200,reg0=0x200000/0x600000 actions=output:NXM_NX_REG1[]",
               ""]
    c = gpc.Classifier()
    n, skipped = c.load_flows(dumped)
    assert n == len(flows) and skipped == 3
    ref = gpc.Classifier()
    ref.load_flows(flows)
    assert normalize_flows(c.dump_flows()) == normalize_flows(ref.dump_flows())


def test_parse_errors_name_the_line():
    c = gpc.Classifier()
    good = BATCH["multiple K8s NetworkPolicy rules"]["expected_flows"][0]
    for bad in ("table=EgressRule, priority=200,ip,nw_src=300.1.1.1 actions=conjunction(1,1/2)",
                "table=EgressRule, priority=200,ip,frobnicate=1 actions=drop",
                "table=EgressRule, priority=200,ip actions=output:3",
                "table=EgressRule, priority=200,ip"):
        with pytest.raises(gpc.GpcError) as e:
            c.load_flows([good, bad])
        assert "line 2" in str(e.value)
    assert c.dump_flows() == []  # nothing applied


def test_loaded_flows_commit_full_builds():
    wl = workload.config1(seed=42)
    src = _compiled(wl)
    c = gpc.Classifier()
    c.load_flows(src.dump_flows())
    emu.commit_host(c)
    c.load_flows(src.dump_flows()[:5], replace=False)
    emu.commit_host(c)
    st = c.image_stats()
    assert st["n_full_builds"] == 2 and st["n_delta_builds"] == 0
