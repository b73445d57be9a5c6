"""Churn path: AddPolicyRuleAddress / DeletePolicyRuleAddress / Uninstall / re-install /
ReassignFlowPriorities applied to the product library and to the oracle in lock step. After every
step the realized flow tables must be identical (network_policy.go:1661-1710, 1570, 1873) and the
committed image (CPU emulation of the kernel body) must give the oracle classifier's verdicts."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import compiler as oc
from oracle import ovs_cls
from tests import emu
from tests.util import normalize_flows

N_PKTS = 300


def _verdicts_oracle(fnp, tiers, cols):
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), tiers)
    out = np.zeros((N_PKTS, 2), dtype=gpc.VERDICT_DTYPE)
    for i in range(N_PKTS):
        e, g = pipe.classify({k: int(v[i]) for k, v in cols.items()})
        for j, v in enumerate((e, g)):
            out[i, j] = (v[1], v[0], v[2], v[3], v[4])
    return out


def _check(clf, fnp, tiers, cols, step):
    got_f, want_f = normalize_flows(clf.dump_flows()), normalize_flows(fnp.dump_flows())
    assert got_f == want_f, "%s: flows differ\nmissing %s\nextra %s" % (step, sorted(want_f - got_f)[:5],
                                                                        sorted(got_f - want_f)[:5])
    emu.commit_host(clf)
    got = emu.classify(clf, cols)
    want = _verdicts_oracle(fnp, tiers, cols)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, "%s: %d mismatches, first %s vs %s" % (step, len(bad), got[bad[0]], want[bad[0]])


def _ip(v):
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


@pytest.mark.parametrize("name,seed", [("C1", 3), ("C3s", 4)])
def test_churn_lockstep(name, seed):
    wl = workload.config1(seed=seed) if name == "C1" else workload.config3(seed=seed, n_policies_per_dir=5,
                                                                              rules_per_policy=6)
    rng = np.random.default_rng(seed)
    rules = copy.deepcopy(wl.rules)
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in rules}
    cols = workload.gen_packets(wl, N_PKTS, seed=seed)
    clf = gpc.Classifier()
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(rules))
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(rules))
    _check(clf, fnp, tiers, cols, "batch")

    by_id = {r["flow_id"]: r for r in rules}
    ids = sorted(by_id)
    done = []
    for step in range(12):
        rid = int(rng.choice(ids))
        r = by_id[rid]
        prio = r.get("priority")
        kind = ["add", "del", "reinstall", "add"][step % 4]
        if kind == "add":
            # peer addresses taken from the packet stream so the new flows are actually hit
            side = "src" if r.get("from") else "dst"
            key = "src" if side == "src" else "dst"
            if side == "dst" and not r.get("to"):
                continue
            pick = rng.choice(N_PKTS, size=3, replace=False)
            addrs = [_ip(int(cols[key][i])) for i in pick]
            clf.add_policy_rule_address(rid, side, addrs, prio)
            fnp.add_policy_rule_address(rid, side, addrs, prio)
            r.setdefault("from" if side == "src" else "to", []).extend(addrs)
        elif kind == "del":
            side = "src" if r.get("from") else "dst"
            lst = r["from"] if side == "src" else r.get("to")
            if not lst or len(lst) < 2:
                continue
            victim = [lst[0]]
            clf.delete_policy_rule_address(rid, side, victim, prio)
            fnp.delete_policy_rule_address(rid, side, victim, prio)
            del lst[0]
        else:
            s1 = clf.uninstall_policy_rule_flows(rid)
            s2 = fnp.uninstall_policy_rule_flows(rid)
            assert sorted(s1) == sorted(s2)
            _check(clf, fnp, tiers, cols, "uninstall %d" % rid)
            clf.install_policy_rule_flows(copy.deepcopy(r))
            fnp.install_policy_rule_flows(copy.deepcopy(r))
        _check(clf, fnp, tiers, cols, "%s %d" % (kind, rid))
        done.append(kind)
    assert {"add", "del", "reinstall"} <= set(done), done


def test_reassign_priorities_lockstep():
    wl = workload.config3(seed=9, n_policies_per_dir=4, rules_per_policy=5)
    rules = copy.deepcopy(wl.rules)
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in rules}
    cols = workload.gen_packets(wl, N_PKTS, seed=9)
    clf = gpc.Classifier()
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(rules))
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(rules))
    for table in ("AntreaPolicyIngressRule", "AntreaPolicyEgressRule"):
        used = sorted({r["priority"] for r in rules if r["table"] == table})
        # swap the order of the two highest rules and move a third to a free slot
        free = max(used) + 7
        upd = {used[-1]: used[-2], used[-2]: used[-1], used[0]: free}
        clf.reassign_flow_priorities(upd, table)
        fnp.reassign_flow_priorities(upd, table)
        _check(clf, fnp, tiers, cols, "reassign %s" % table)
