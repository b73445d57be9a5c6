"""IPv6 delta epochs (image.cpp extend_image6 + the IPv6 journal).

A seeded churn log (tests/golden/make_churn_fixture.py's op mix: address adds / deletes incl. the
base image's own peers, uninstall / reinstall, ReassignFlowPriorities, a commit every 100 ops)
is mapped into fd00:10::/96 and replayed on an IPv6 (and a dual-stack) context, and the IPv4 log
on an IPv4 context. After every commit the IPv6 image's emulated verdicts (tests/csrc/emu.cpp,
the kernel body over base + journal) equal the IPv4 image's on the same packets embedded the same
way -- metamorphic parity, the IPv4 side being pinned by the oracles (test_churn.py, the C5
fixture). At the end the IPv6 verdicts are also checked against the Python oracle directly, and
a compaction (full rebuild) gives the same verdicts. The commits must have gone through the
delta path (new prefixes interned in place, rules appended to the IPv6 journal)."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from tests import emu
from tests.golden import make_churn_fixture as mcf
from tests.test_emu_parity import _cmp

N_OPS = 500


def _wl():
    return workload.config3(seed=11, n_policies_per_dir=6, rules_per_policy=8)


def _rule6(r, dual):
    r6 = copy.deepcopy(r)
    for side in ("from", "to"):
        if r.get(side) is not None:
            mapped = [workload._v6_addr(a) for a in r[side]]
            r6[side] = (list(r[side]) + [m for m, a in zip(mapped, r[side]) if m != a]) if dual else mapped
    return r6


def _map_log(log, dual):
    """The op log with its IPv4 addresses embedded in fd00:10::/96 (dual: both families)."""
    out = []
    for o in log:
        o = copy.deepcopy(o)
        if o["op"] in ("add", "del"):
            v6 = [workload._v6_addr(a) for a in o["addrs"]]
            o["addrs"] = (o["addrs"] + [m for m, a in zip(v6, o["addrs"]) if m != a]) if dual else v6
        elif o["op"] == "install":
            o["rule"] = _rule6(o["rule"], dual)
        out.append(o)
    return out


def _packets(wl, log, n, seed):
    """Workload packets, a third of them re-addressed to peers the log adds."""
    cols = workload.gen_packets(wl, n, seed=seed)
    added = [int.from_bytes(bytes(int(x) for x in a.split(".")), "big")
             for o in log if o["op"] == "add" for a in o["addrs"] if isinstance(a, str) and "." in a and "/" not in a]
    if added:
        rng = np.random.default_rng(seed)
        pick = rng.random(n) < 0.33
        side = rng.random(n) < 0.5
        vals = np.array(added, np.uint32)[rng.integers(len(added), size=n)]
        cols["src"] = np.where(pick & side, vals, cols["src"]).astype(np.uint32)
        cols["dst"] = np.where(pick & ~side, vals, cols["dst"]).astype(np.uint32)
    return cols


def _ctx(rules, ipv4, ipv6):
    c = gpc.Classifier(ipv4=ipv4, ipv6=ipv6, compact_after=-1)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(rules))
    emu.commit_host(c)
    return c


@pytest.mark.parametrize("dual", [False, True], ids=["v6", "dual"])
def test_ipv6_delta_epochs_track_ipv4(dual):
    wl = _wl()
    log4 = mcf.ops(wl, seed=0x6D)[:N_OPS] + [{"op": "commit"}]
    log6 = _map_log(log4, dual)
    cols = _packets(wl, log4, 3000, seed=12)
    cols6 = workload.packets_to_v6(cols)
    c4 = _ctx(wl.rules, True, False)
    c6 = _ctx(workload.to_ipv6(wl, dual=dual).rules, dual, True)
    s0 = c6.image_stats()
    assert s0["v6_full_builds"] == 1 and s0["v6_delta_builds"] == 0
    commits = [0]

    def check():
        emu.commit_host(c4)
        emu.commit_host(c6)
        commits[0] += 1
        want = emu.classify(c4, cols)
        _cmp(emu.classify6(c6, cols6), want, cols)
        if dual:
            _cmp(emu.classify(c6, cols), want, cols)

    # replay both logs commit by commit (the commit markers sit at the same positions)
    i4 = iter(log4)
    for o6 in log6:
        o4 = next(i4)
        if o6["op"] == "commit":
            check()
            continue
        mcf.apply(c4, [o4])
        mcf.apply(c6, [o6])
    st = c6.image_stats()
    assert commits[0] >= 5
    assert st["v6_delta_builds"] >= commits[0] - 1 and st["v6_full_builds"] <= 2, st
    assert st["v6_overlay_rules"] > 0 and st["v6_prefixes"] > s0["v6_prefixes"], st
    # the final epoch against the oracle directly, then a full rebuild gives the same verdicts
    n = 300
    sub = {k: v[:n] for k, v in cols6.items()}
    _cmp(emu.classify6(c6, sub), _oracle_after(workload.to_ipv6(wl, dual=dual).rules, log6, sub, n, dual), sub)
    before = emu.classify6(c6, cols6)
    emu.commit_host(c6, full=True)
    assert c6.image_stats()["v6_overlay_rules"] == 0
    _cmp(emu.classify6(c6, cols6), before, cols)


def _oracle_after(rules, log, cols6, n, dual):
    """Python oracle verdicts of the IPv6 packets after the oracle compiler replayed the log."""
    from oracle import compiler as oc
    from oracle import ovs_cls
    fnp = oc.FeatureNetworkPolicy(ipv4=dual, ipv6=True)
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(rules))
    mcf.apply(fnp, log)
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), {r["flow_id"]: int(r.get("tier_priority") or 0) for r in rules})
    out = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for i in range(n):
        pkt = {k: int(v[i]) for k, v in cols6.items() if v.ndim == 1}
        for k in ("src6", "dst6"):
            pkt[k[:-1]] = int.from_bytes(bytes(cols6[k][i]), "big")
        pkt["eth"] = 0x86DD
        e, g = pipe.classify(pkt)
        for j, v in enumerate((e, g)):
            out[i, j] = (v[1], v[0], v[2], v[3], v[4])
    return out


def _hit_packets(r, srcs):
    """IPv6 packets from `srcs` that match every clause of ingress rule r but its From."""
    import ipaddress
    n = len(srcs)
    svc = r["service"][0]
    proto = {"TCP": 6, "UDP": 17}[svc["protocol"]]
    return {"src6": np.array([list(ipaddress.ip_address(a).packed) for a in srcs], np.uint8),
            "dst6": np.tile(np.frombuffer(ipaddress.ip_address("fd00:10::a00:5").packed, np.uint8), (n, 1)),
            "sport": np.full(n, 40000, np.uint16), "dport": np.full(n, svc["port"], np.uint16),
            "proto": np.full(n, proto, np.uint8), "out_port": np.full(n, r["to"][0]["ofport"], np.uint32)}


def test_new_prefix_lengths_are_incremental():
    """a delta epoch that brings prefix lengths the base LPM does not search
    interns them in place (up to kV6MaxNewLens = 3 new lengths, leaves probed in the journal's
    overflow hash after the binary search): no IPv6 rebuild, verdicts == the Python oracle for
    addresses inside and next to the new prefixes. A fourth new length, or a prefix below a leaf
    added since the base, rebuilds the IPv6 image (and the verdicts stay right)."""
    wl = _wl()
    rules6 = workload.to_ipv6(wl).rules
    c6 = _ctx(rules6, False, True)
    r = next(r for r in rules6 if r["direction"] == "In" and r.get("from") and r["action"] == "Allow")
    log = []

    def add(addr):
        o = {"op": "add", "fid": r["flow_id"], "side": "src", "addrs": [addr], "priority": r.get("priority")}
        mcf.apply(c6, [o])
        log.append(o)
        emu.commit_host(c6)
        return c6.image_stats()

    full0 = c6.image_stats()["v6_full_builds"]
    lens = {int(a["ipnet"].split("/")[1]) for rr in rules6 for side in ("from", "to") for a in rr.get(side) or []
            if isinstance(a, dict) and "ipnet" in a}
    new = [L for L in (47, 61, 77, 93) if L not in lens]
    assert len(new) == 4
    nets = ["2001:db8:1234::/%d" % new[0], "2001:db8:5678::/%d" % new[1], "2001:db9::/%d" % new[2]]
    for k, net in enumerate(nets):
        st = add({"ipnet": net})
        assert st["v6_full_builds"] == full0 and st["v6_delta_builds"] == k + 1, (net, st)
    srcs = ["2001:db8:1234::1", "2001:db8:1235::1", "2001:db8:5678::9", "2001:db8:5679::9", "2001:db9::42",
            "2001:db9:0:1::1", "2001:db7::1", "fd00:10::a00:1"]
    cols6 = _hit_packets(r, srcs)
    want = _oracle_after(rules6, log, cols6, len(srcs), False)
    got = emu.classify6(c6, cols6)
    _cmp(got, want, cols6)
    assert (got[:, 1]["conj_id"] == r["flow_id"]).sum() >= 3
    # a fourth new length: full rebuild
    st = add({"ipnet": "2001:dba::/%d" % new[3]})
    assert st["v6_full_builds"] == full0 + 1
    # below a leaf interned since the (new) base: full rebuild again
    st = add({"ipnet": "2001:dbb::/%d" % new[0]})
    assert st["v6_full_builds"] == full0 + 1
    st = add({"ipnet": "2001:dbb::/%d" % (new[0] + 16)})
    assert st["v6_full_builds"] == full0 + 2
    srcs += ["2001:dba::5", "2001:dbb::1", "2001:dbb:1::1"]
    cols6 = _hit_packets(r, srcs)
    _cmp(emu.classify6(c6, cols6), _oracle_after(rules6, log, cols6, len(srcs), False), cols6)