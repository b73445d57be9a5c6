"""GPU tier: IPv6 delta epochs on the device. A dual-stack context replays
the seeded churn log (tests/test_ipv6_delta.py: address adds / deletes, uninstall / reinstall,
priority reassignment, mapped into fd00:10::/96 next to the IPv4 addresses) through delta
commits. After each commit the device's IPv6 verdicts (gpc_classify6 over the base image + the
IPv6 journal + its overflow LPM table) equal the host emulation of the same epoch, which the CPU
tier pins to the IPv4 image and to the oracle; at the end the device is checked against the
Python oracle directly, and after a compaction again."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from tests import emu
from tests.golden import make_churn_fixture as mcf
from tests.test_emu_parity import _cmp
from tests.test_ipv6_delta import _map_log, _oracle_after, _packets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


@pytest.mark.parametrize("size", ["small", "C3-10k"])
def test_gpu_ipv6_delta_epochs_dual_stack(size):
    wl = (workload.config3(seed=11, n_policies_per_dir=6, rules_per_policy=8) if size == "small"
          else workload.config3(n_policies_per_dir=50, rules_per_policy=100))
    n_ops = 600 if size == "small" else 1500
    log4 = mcf.ops(wl, seed=0x6D)[:n_ops] + [{"op": "commit"}]
    log6 = _map_log(log4, dual=True)
    cols = _packets(wl, log4, 20000 if size == "small" else 100_000, seed=13)
    cols6 = workload.packets_to_v6(cols)
    c = gpc.Classifier(ipv4=True, ipv6=True, compact_after=-1)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(workload.to_ipv6(wl, dual=True).rules))
    c.commit()
    checked = 0
    for k, o in enumerate(log6):
        if o["op"] != "commit":
            mcf.apply(c, [o])
            continue
        c.commit()
        if checked < 4 or o is log6[-1]:
            _cmp(c.classify6_host(cols6), emu.classify6(c, cols6), cols)
            _cmp(c.classify_host(cols), emu.classify(c, cols), cols)
            checked += 1
    st = c.image_stats()
    assert st["v6_delta_builds"] >= 5 and st["v6_overlay_rules"] > 0, st
    got = c.classify6_host(cols6)
    if size == "small":
        n = 300
        sub = {k: v[:n] for k, v in cols6.items()}
        _cmp(got[:n], _oracle_after(workload.to_ipv6(wl, dual=True).rules, log6, sub, n, True), sub)
    else:
        # at the C3-10k size the device's IPv6 verdicts of the last delta epoch
        # against the C oracle, every packet: the oracle compiler replays the IPv4 log over the IPv4
        # rules and the C classifier runs the IPv4 packets (the fd00:10::/96 embedding preserves every
        # match); the dual-stack context's IPv4 verdicts must equal them too
        from oracle import compiler as oc
        from oracle import parity
        fnp = oc.FeatureNetworkPolicy()
        fnp.initialize()
        fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        mcf.apply(fnp, log4)
        want = parity.oracle_pipeline(wl, flows=fnp.dump_flows()).classify(cols)
        for fam, v in (("IPv6", got), ("IPv4", c.classify_host(cols))):
            res = parity.compare(v, want)
            assert res["mismatches"] == 0, (fam, res)
    c.compact()
    assert c.image_stats()["v6_overlay_rules"] == 0
    _cmp(c.classify6_host(cols6), got, cols)


def test_gpu_upload_failure_then_delta_resyncs():
    """a commit that rebuilds the host bases in full and then fails to upload
    them must not leave the device extending a stale (or missing) base. After an injected upload
    failure on a full rebuild, the next delta commit re-uploads both bases and the whole journals;
    the device's IPv4 and IPv6 verdicts then equal the host emulation of the epoch."""
    wl = workload.config3(seed=11, n_policies_per_dir=6, rules_per_policy=8)
    log4 = mcf.ops(wl, seed=0x6E)[:300]
    log6 = _map_log(log4 + [{"op": "commit"}], dual=True)[:-1]
    cols = _packets(wl, log4, 20000, seed=17)
    cols6 = workload.packets_to_v6(cols)
    c = gpc.Classifier(ipv4=True, ipv6=True, compact_after=-1)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(workload.to_ipv6(wl, dual=True).rules))
    c.commit()
    mcf.apply(c, [o for o in log6[:100] if o["op"] != "commit"])
    c.commit()  # a delta epoch on both families
    mcf.apply(c, [o for o in log6[100:150] if o["op"] != "commit"])
    c.debug_fail_uploads(1)
    with pytest.raises(gpc.GpcError):
        c.compact()  # full rebuild of both host bases; the device keeps the previous epoch
    c.debug_fail_uploads(0)
    mcf.apply(c, [o for o in log6[150:] if o["op"] != "commit"])
    c.commit()  # delta over the new host bases: every slot must re-upload them first
    assert c.image_stats()["v6_overlay_rules"] > 0
    _cmp(c.classify6_host(cols6), emu.classify6(c, cols6), cols)
    _cmp(c.classify_host(cols), emu.classify(c, cols), cols)


def test_gpu_new_prefix_lengths_incremental():
    """New IPv6 prefix lengths in a delta epoch (core.hpp v6_codes: probes of the new lengths after
    the binary search) on the device: no IPv6 rebuild, device == emulation == Python oracle."""
    from tests.test_ipv6_delta import _hit_packets, _oracle_after
    wl = workload.config3(seed=11, n_policies_per_dir=6, rules_per_policy=8)
    rules6 = workload.to_ipv6(wl).rules
    c = gpc.Classifier(ipv4=False, ipv6=True, compact_after=-1)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(rules6))
    c.commit()
    r = next(r for r in rules6 if r["direction"] == "In" and r.get("from") and r["action"] == "Allow")
    log = [{"op": "add", "fid": r["flow_id"], "side": "src", "addrs": [{"ipnet": net}], "priority": r.get("priority")}
           for net in ("2001:db8:1234::/47", "2001:db8:5678::/61", "2001:db9::/77")]
    full0 = c.image_stats()["v6_full_builds"]
    for o in log:
        mcf.apply(c, [o])
        c.commit()
    assert c.image_stats()["v6_full_builds"] == full0
    srcs = ["2001:db8:1234::1", "2001:db8:1235::1", "2001:db8:5678::9", "2001:db8:5679::9", "2001:db9::42",
            "2001:db9:0:1::1", "2001:db7::1", "fd00:10::a00:1"] * 40
    cols6 = _hit_packets(r, srcs)
    got = c.classify6_host(cols6)
    _cmp(got, emu.classify6(c, cols6), cols6)
    n = 8
    sub = {k: v[:n] for k, v in cols6.items()}
    _cmp(got[:n], _oracle_after(rules6, log, sub, n, False), sub)
    assert (got[:, 1]["conj_id"] == r["flow_id"]).sum() >= 3 * 40
