"""GPU tier: the HIP path (gpc_classify through the C-ABI) against the oracle."""
import copy
import ipaddress

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import compiler as oc
from oracle import ovs_cls
from tests import emu
from tests.test_emu_parity import WORKLOADS, _cmp, oracle_verdicts
from tests.util import assign_tables, load_golden

pytestmark = pytest.mark.gpu

ACT = {"NONE": 0, "NO_MATCH": 1, "ALLOW": 2, "DROP": 3, "REJECT": 4, "ISOLATION_DROP": 5, "BYPASS": 6}


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


def _gpu(rules, cols, count=False, init=True):
    c = gpc.Classifier()
    if init:
        c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(rules))
    c.commit()
    return c.classify_host(cols, count=count), c


def test_appendix_a_known_answers():
    batch = {c["name"]: c for c in load_golden("np_batch_install.json")["cases"]}
    for s in load_golden("appendix_a.json")["sets"]:
        rules = assign_tables(copy.deepcopy(batch[s["flows_from_case"]]["rules"]))
        pk = [tc["pkt"] for tc in s["packets"]]
        cols = {k: np.array([int(ipaddress.ip_address(p[k])) if k in ("src", "dst") else int(p.get(k, 0)) for p in pk])
                for k in ("src", "dst", "proto", "sport", "dport", "out_port", "tun_id")}
        got, _ = _gpu(rules, cols)
        for i, tc in enumerate(s["packets"]):
            for j, key in enumerate(("egress", "ingress")):
                a, conj, table, flags = tc[key]
                v = got[i, j]
                assert (v["action"], v["conj_id"], v["table"], v["flags"]) == (ACT[a], conj, table, flags), (tc, key, v)


@pytest.mark.parametrize("name", sorted(WORKLOADS))
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_vs_oracle(name, seed):
    wl = WORKLOADS[name](seed)
    n = 500
    cols = workload.gen_packets(wl, n, seed=seed)
    want, _ = oracle_verdicts(wl.rules, cols, n)
    got, _ = _gpu(wl.rules, cols)
    _cmp(got, want, cols)


def test_gpu_counters_match_oracle_metrics():
    wl = workload.config1(seed=5)
    n = 600
    cols = workload.gen_packets(wl, n, seed=5)
    u = np.random.default_rng(5).random(n)  # +new+trk / +trk (-new: no session) / +est+trk (bypass)
    cols["ct_state"] = np.where(u < 0.7, 0x21, np.where(u < 0.9, 0x20, 0x22)).astype(np.uint8)
    want, pipe = oracle_verdicts(wl.rules, cols, n)
    d = pipe.metric_dumps()
    want_m = oc.network_policy_metrics(d["EgressMetric"], d["IngressMetric"])
    got, c = _gpu(wl.rules, cols, count=True)
    _cmp(got, want, cols)
    got_m = c.network_policy_metrics()
    assert {k: v for k, v in got_m.items()} == {k: v for k, v in want_m.items()}


def test_gpu_matches_image_emulation_large():
    """Full C3 (100k rules): device result == host emulation of the same image on 200k packets."""
    wl = workload.config3()
    cols = workload.gen_packets(wl, 200_000, seed=11)
    got, c = _gpu(wl.rules, cols)
    want = emu.classify(c, cols)
    _cmp(got, want, cols)
