"""gpc_trace (SURVEY §5 Traceflow readback, traceflow/packetin.go:211-270; ofproto/trace,
ovsctl.go:91-183): per packet, the rule tables its walk evaluated with each table's decision
(verdict, flags, deciding conjunction, flow priority). The table sequence and decisions equal the
oracle's own walk of the same flows (ovs_cls.Pipeline.classify(trace=...)), and the final verdict
equals gpc_classify's. CPU tier through the emulated walk; GPU tier through the device trace."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import compiler as oc
from oracle import ovs_cls
from tests import emu


def _setup(wl, dns=False):
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.initialize()
        side.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        if dns:
            side.new_dns_packet_in_conjunction(9999)
            side.add_address_to_dns_conjunction(9999, ["%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)
                                                       for v in (int(x) for x in wl.local_ips[:5])])
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    return ovs_cls.Pipeline(fnp.dump_flows(), tiers), c


def _packets(wl, n, seed):
    cols = workload.gen_packets(wl, n, seed=seed)
    rng = np.random.default_rng(seed)
    cols["ct_state"] = rng.choice([0x21, 0x21, 0x21, 0x22, 0x28], n).astype(np.uint8)
    return cols


def _check(pipe, c, cols, tracer, n):
    kinds = set()
    for i in range(n):
        pkt = {k: int(v[i]) for k, v in cols.items()}
        want = []
        e, g = pipe.classify(dict(pkt), trace=want)
        verdicts, steps = tracer(c, pkt)[:2]
        got = [(s["table"], s["verdict"], s["flags"], s["conj_id"], s["priority"]) for s in steps]
        assert got == want, (pkt, got, want)
        for j, v in enumerate((e, g)):
            assert tuple(verdicts[j][["action", "conj_id", "table", "tier", "flags"]].item()) == v, (pkt, verdicts, e, g)
        kinds |= {s[1] for s in want}
    return kinds


@pytest.mark.parametrize("name", ["C1", "C3s"])
def test_trace_emu_vs_oracle(name):
    wl = workload.config1(seed=7) if name == "C1" else workload.config3(seed=7, n_policies_per_dir=6, rules_per_policy=8)
    pipe, c = _setup(wl, dns=name == "C1")
    emu.commit_host(c)
    kinds = _check(pipe, c, _packets(wl, 300, 7), emu.trace, 300)
    assert {1, 2} <= kinds


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C1", "C3s"])
def test_trace_device_vs_oracle(name):
    from antrea_amd.build import build
    build()
    wl = workload.config1(seed=8) if name == "C1" else workload.config3(seed=8, n_policies_per_dir=6, rules_per_policy=8)
    pipe, c = _setup(wl, dns=name == "C1")
    c.commit()
    cols = _packets(wl, 200, 8)
    kinds = _check(pipe, c, cols, lambda c, p: c.trace(p), 200)
    assert {1, 2} <= kinds
    got = c.classify_host(cols)  # the traced verdicts are the data path's
    for i in range(20):
        assert (c.trace({k: int(v[i]) for k, v in cols.items()})[0] == got[i]).all()
