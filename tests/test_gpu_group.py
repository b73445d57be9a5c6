"""GPU tier: the packet grouping pre-pass of gpc_classify (classify.hip group_*: counting sort of
every tile of the batch by a key -- the scan lengths of both policy stages, or the top byte of
nw_src -- classification in grouped order, verdicts and LB results scattered back to caller order)
is invisible in the results: verdicts, LB results and per-rule counters equal the ungrouped
launch's exactly, for both keys, for ragged batch sizes around the 16384-packet tile and with every
optional packet column present."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


KEYS = [gpc.GROUP_KEY_SCAN, gpc.GROUP_KEY_ADDR]


def _pair(wl, services=False, keys=(gpc.GROUP_KEY_SCAN,)):
    """[plain, grouped with each key...]"""
    out = []
    for g, k in [(-1, 0)] + [(1, k) for k in keys]:
        c = gpc.Classifier(group_packets=g, group_key=k)
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        if services:
            workload.install_services(c, wl)
        c.commit()
        out.append(c)
    return out


def _metrics(c):
    return {k: v for k, v in c.network_policy_metrics().items() if any(v)}


def _optional_columns(cols, rng):
    n = len(cols["src"])
    cols = dict(cols)
    cols["in_port"] = rng.integers(0, 200, n).astype(np.uint32)
    cols["tun_id"] = rng.integers(0, 4, n).astype(np.uint32)
    cols["ct_src"] = np.where(rng.random(n) < 0.9, cols["src"], rng.integers(0, 1 << 32, n)).astype(np.uint32)
    cols["ct_dst"] = np.where(rng.random(n) < 0.9, cols["dst"], rng.integers(0, 1 << 32, n)).astype(np.uint32)
    cols["ct_state"] = rng.choice([0x21, 0x22, 0x24, 0x2a], size=n, p=[0.7, 0.2, 0.05, 0.05]).astype(np.uint8)
    cols["dest"] = rng.choice(4, size=n, p=[0.85, 0.05, 0.05, 0.05]).astype(np.uint8)
    cols["ct_mark"] = np.where(rng.random(n) < 0.05, 0x40, 0).astype(np.uint8)
    cols["svc_group"] = np.where(rng.random(n) < 0.1, rng.integers(1, 50, n), 0).astype(np.uint32)
    return cols


@pytest.mark.parametrize("key", KEYS)
@pytest.mark.parametrize("n", [1, 63, 16383, 16384, 16385, 3 * 16384 + 5, (1 << 18) + 7])
def test_grouped_equals_plain_ragged(n, key):
    wl = workload.config1(seed=9)
    cols = workload.gen_packets(wl, n, seed=9)
    plain, grouped = _pair(wl, keys=(key,))
    a = plain.classify_host(cols, count=True)
    b = grouped.classify_host(cols, count=True)
    assert (a == b).all()
    assert _metrics(plain) == _metrics(grouped)


def test_grouped_equals_plain_optional_columns_c3():
    """C3's rule shapes at a fifth of its size (20k rules: the builds dominate the test time; the
    full-size grouped path is checked against the oracle in test_gpu_fullscale.py)."""
    wl = workload.config3(n_policies_per_dir=100)
    rng = np.random.default_rng(12)
    n = 150_000
    cols = _optional_columns(workload.gen_packets(wl, n, seed=12), rng)
    plain, *grouped = _pair(wl, keys=KEYS)
    a = plain.classify_host(cols, count=True)
    for g in grouped:
        b = g.classify_host(cols, count=True)
        assert (a == b).all()
        assert _metrics(plain) == _metrics(g)
    assert len(np.unique(a["action"])) >= 4


def test_grouped_equals_plain_c2_lane_sort(monkeypatch):
    """C2: the plain launch regroups lanes inside each block (lane-sort kernels, forced: since round
    6 no benchmark configuration reaches the auto bar); the scan-key grouped launch runs the plain
    kernels over tiles already ordered by scan length."""
    monkeypatch.setenv("GPC_LANE_SORT", "1")
    wl = workload.config2()
    n = 200_000
    cols = workload.gen_packets(wl, n, seed=14)
    plain, *grouped = _pair(wl, keys=KEYS)
    a = plain.classify_host(cols, count=True)
    for g in grouped:
        b = g.classify_host(cols, count=True)
        assert (a == b).all()
        assert _metrics(plain) == _metrics(g)


def test_grouped_equals_plain_services_lb():
    from tests.test_service import _svc_workload
    wl = _svc_workload("C1", 61)
    n = 50_000
    cols = workload.gen_packets(wl, n, seed=13)
    plain, *grouped = _pair(wl, services=True, keys=KEYS)
    a, la = plain.classify_host(cols, count=True, lb=True)
    assert ((la["flags"] & gpc.LB_HIT) != 0).any()
    for g in grouped:
        b, lbb = g.classify_host(cols, count=True, lb=True)
        assert (a == b).all() and (la == lbb).all()
        assert _metrics(plain) == _metrics(g)


def test_grouped_device_stream_batch():
    """Device-pointer path on a torch stream with a grouped batch (>= 2^18 packets) equals an
    ungrouped one (20k C3-shaped rules; auto mode no longer groups against composite images, so the
    grouped run is forced)."""
    import torch
    wl = workload.config3(n_policies_per_dir=100)
    n = 1 << 19
    cols = workload.gen_packets_torch(wl, n, device="cuda")
    outs = []
    for g in (1, -1):
        c = gpc.Classifier(group_packets=g)
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        c.commit()
        out = torch.zeros(2 * n * 8, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        c.classify_device(gpc.pkt_soa_device(cols), n, out.data_ptr(), count=True, stream=s.cuda_stream)
        s.synchronize()
        outs.append((out.cpu(), _metrics(c)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]


def test_batch_over_launch_limit_is_einval():
    """n > GPC_MAX_BATCH (2^32 - 256) is rejected with -GPC_EINVAL before any allocation or launch
    (the grouping scratch for such a batch would not be allocated either)."""
    import ctypes as C
    import torch
    wl = workload.config3(n_policies_per_dir=5, rules_per_policy=10)
    c = gpc.Classifier(group_packets=1)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    c.commit()
    cols = workload.gen_packets_torch(wl, 256, device="cuda")
    out = torch.zeros(2 * 256 * 8, dtype=torch.uint8, device="cuda")
    soa = gpc.pkt_soa_device(cols)
    for n in ((1 << 32) - 255, 1 << 32, (1 << 40)):
        rc = c.lib.gpc_classify(c.h, C.byref(soa), C.c_size_t(n), C.c_void_p(out.data_ptr()), 0, None)
        assert rc == -gpc.GPC_EINVAL, (n, rc)
    c.classify_device(soa, 256, out.data_ptr(), count=False, stream=0)
    torch.cuda.synchronize()


def test_grouped_many_streams():
    """Grouped batches on more streams than the scratch cache keeps (8): idle buffers of finished
    streams are released, results stay identical to the plain launch."""
    import torch
    wl = workload.config1(seed=21)
    n = 20_000
    cols = workload.gen_packets_torch(wl, n, device="cuda")
    soa = gpc.pkt_soa_device(cols)
    ref = torch.zeros(2 * n * 8, dtype=torch.uint8, device="cuda")
    plain = gpc.Classifier(group_packets=-1)
    grouped = gpc.Classifier(group_packets=1)
    for c in (plain, grouped):
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        c.commit()
    plain.classify_device(soa, n, ref.data_ptr(), stream=0)
    torch.cuda.synchronize()
    outs = []
    for k in range(12):
        s = torch.cuda.Stream()
        o = torch.zeros_like(ref)
        grouped.classify_device(soa, n, o.data_ptr(), stream=s.cuda_stream)
        outs.append((s, o))
        if k % 3 == 2:
            s.synchronize()
    torch.cuda.synchronize()
    for s, o in outs:
        assert torch.equal(o, ref)


@pytest.mark.parametrize("n", [1, 16383, 16385, 3 * 16384 + 5])
def test_grouped_ipv6_equals_plain(n):
    """IPv6 batches (gpc_classify6): grouped == plain, verdicts and counters, with ct_*6 columns
    (the code launch maps four address columns; grouping runs over the code columns)."""
    wl = workload.config1(seed=9)
    w6 = workload.to_ipv6(wl, dual=True)
    rng = np.random.default_rng(n)
    cols = workload.packets_to_v6(workload.gen_packets(wl, n, seed=9))
    cols["ct_src6"] = np.ascontiguousarray(np.where((rng.random(n) < 0.9)[:, None], cols["src6"], cols["dst6"]))
    res = []
    for g in (-1, 1):
        c = gpc.Classifier(ipv4=True, ipv6=True, group_packets=g)
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(w6.rules))
        c.commit()
        res.append((c.classify6_host(cols, count=True), _metrics(c)))
    assert (res[0][0] == res[1][0]).all()
    assert res[0][1] == res[1][1]


def test_grouped_per_thread_default_stream_two_threads():
    """hipStreamPerThread (handle 2) names a different stream on every host thread: two threads
    classifying grouped batches on it at the same time get separate grouping scratch (keyed by
    stream and thread), so their verdicts equal the plain launch's."""
    import threading
    import torch
    HIP_STREAM_PER_THREAD = 2
    wl = workload.config3(n_policies_per_dir=20, rules_per_policy=50)
    n = 1 << 18
    colsets = [workload.gen_packets_torch(wl, n, device="cuda", seed=s) for s in (31, 32)]
    plain = gpc.Classifier(group_packets=-1)
    grouped = gpc.Classifier(group_packets=1)
    for c in (plain, grouped):
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        c.commit()
    refs = []
    for cols in colsets:
        r = torch.zeros(2 * n * 8, dtype=torch.uint8, device="cuda")
        plain.classify_device(gpc.pkt_soa_device(cols), n, r.data_ptr(), stream=0)
        refs.append(r)
    torch.cuda.synchronize()
    outs = [[torch.zeros_like(refs[0]) for _ in range(4)] for _ in colsets]
    errs = []

    def work(k):
        try:
            soa = gpc.pkt_soa_device(colsets[k])
            for o in outs[k]:
                grouped.classify_device(soa, n, o.data_ptr(), stream=HIP_STREAM_PER_THREAD)
            assert grouped.stream_epoch(HIP_STREAM_PER_THREAD) > 0  # keyed by this thread
        except Exception as e:  # reported by the main thread
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for k in range(2):
        for o in outs[k]:
            assert torch.equal(o, refs[k])


@pytest.mark.parametrize("group", [-1, 1], ids=["plain", "grouped"])
def test_service_split_equals_single_launch(group, monkeypatch):
    """GPC_SVC_SPLIT=1 (read at gpc_create): Service batches as two launches, the DNAT'ed fields
    parked between them, give the same verdicts, LB results and counters as the one-launch default."""
    from tests.test_service import _svc_workload
    wl = _svc_workload("C1", 62)
    n = 40_000
    cols = workload.gen_packets(wl, n, seed=15)
    res = []
    for split in ("0", "1"):
        monkeypatch.setenv("GPC_SVC_SPLIT", split)
        c = gpc.Classifier(group_packets=group)
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        workload.install_services(c, wl)
        c.commit()
        v, lb = c.classify_host(cols, count=True, lb=True)
        res.append((v, lb, _metrics(c)))
    assert ((res[0][1]["flags"] & gpc.LB_HIT) != 0).any()
    assert (res[0][0] == res[1][0]).all() and (res[0][1] == res[1][1]).all()
    assert res[0][2] == res[1][2]
