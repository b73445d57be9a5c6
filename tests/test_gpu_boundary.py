"""GPU tier for the boundary, concurrency and multi-GPU plumbing rows:

* DNS interception (NewDNSPacketInConjunction trio) and the IngressSecurityClassifier bypasses on
  the device, against the oracle's walk of the same flows;
* delta epochs with lane regrouping forced on (the classify_kernel<journal, sorted lanes>
  instantiations), against the host emulation of the same epoch, verdicts and counters;
* classification concurrent with commits (config C5's shape): a control thread publishes delta
  epochs while launches queue on another stream; every launch is bound to exactly one epoch
  (gpc_stream_epoch) and its verdicts equal the emulation of that epoch's snapshot;
* the RCCL counter all-reduce on a world-size-1 NCCL(RCCL) group over the library's device
  counters wrapped zero-copy (the >1 guard of dist.allreduce_counters bypassed)."""
import copy
import os
import socket
import threading
import time

import numpy as np
import pytest

from antrea_amd import gpc, workload
from oracle import compiler as oc
from oracle import ovs_cls
from tests import emu
from tests.test_emu_parity import _cmp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


def _oracle(flows, cols, tiers=None):
    pipe = ovs_cls.Pipeline(flows, tiers or {})
    n = len(cols["src"])
    out = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for i in range(n):
        e, g = pipe.classify({k: int(v[i]) for k, v in cols.items()})
        for j, v in enumerate((e, g)):
            out[i, j] = (v[1], v[0], v[2], v[3], v[4])
    return out


def test_gpu_dns_interception():
    from tests.test_boundary_np import _dns_cols
    wl = workload.config1(seed=12)
    ips = [int(x) for x in wl.local_ips[:5]]
    addrs = ["%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255) for v in ips]
    fnp, c = oc.FeatureNetworkPolicy(), gpc.Classifier()
    for side in (fnp, c):
        side.initialize()
        side.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        side.new_dns_packet_in_conjunction(9999)
        side.add_address_to_dns_conjunction(9999, addrs)
    c.commit()
    cols = _dns_cols(3000, np.random.default_rng(14), np.array(ips, np.uint32))
    got = c.classify_host(cols)
    _cmp(got, _oracle(fnp.dump_flows(), cols), cols)
    assert ((got[:, 1]["flags"] & gpc.VFLAG_PACKETIN) != 0).sum() > 100
    for side in (fnp, c):  # DeleteAddressFromDNSConjunction, published as a delta epoch
        side.delete_address_from_dns_conjunction(9999, addrs[:2])
    c.commit()
    _cmp(c.classify_host(cols), _oracle(fnp.dump_flows(), cols), cols)


@pytest.mark.parametrize("k8s", [True, False])
def test_gpu_ingress_classifier(k8s):
    wl = workload.config1(seed=13)
    n = 3000
    cols = workload.gen_packets(wl, n, seed=15)
    rng = np.random.default_rng(15)
    cols["dest"] = rng.choice([0, 0, 1, 2, 3], n).astype(np.uint8)
    cols["ct_mark"] = np.where(rng.random(n) < 0.25, 0x40, rng.choice([0, 0x10, 0x20], n)).astype(np.uint8)
    fnp, c = oc.FeatureNetworkPolicy(k8s_node=k8s), gpc.Classifier(k8s_node=k8s)
    for side in (fnp, c):
        side.initialize()
        side.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    c.commit()
    got = c.classify_host(cols, count=True)
    _cmp(got, _oracle(fnp.dump_flows(), cols), cols)
    assert ((got[:, 1]["action"] == 6).sum() > n // 4) == k8s


@pytest.mark.parametrize("ext", [1, 0], ids=["extensions", "journal_only"])
def test_gpu_lane_sort_delta_epochs(monkeypatch, ext):
    """GPC_LANE_SORT=1 read at commit: the lane-regrouping kernels run on delta epochs (journal +
    tombstones + sorted lanes, the stage-2 live prefilter included; with point extensions the
    added addresses are extensions of base records beside the uninstalls' tombstones); verdicts
    and counters equal the host emulation of the same epoch."""
    monkeypatch.setenv("GPC_LANE_SORT", "1")
    if not ext:
        monkeypatch.setenv("GPC_NO_EXTENSIONS", "1")
    wl = workload.config3(n_policies_per_dir=20, rules_per_policy=50)
    n = 60000
    cols = workload.gen_packets(wl, n, seed=41)
    rules = copy.deepcopy(wl.rules)
    c = gpc.Classifier()
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(rules))
    c.commit()
    rng = np.random.default_rng(41)
    live = list(rules)
    for step in range(10):
        r = live.pop(int(rng.integers(len(live))))
        side = "src" if r.get("from") else "dst"
        addrs = ["%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 4)) for _ in range(6)]
        addrs += [emu_ip(int(cols[side][i])) for i in rng.choice(n, 6, replace=False)]
        c.add_policy_rule_address(r["flow_id"], side, addrs, r.get("priority"))
        if step % 3 == 2:
            c.uninstall_policy_rule_flows(r["flow_id"])
        else:
            live.append(r)
        c.commit()
    st = c.image_stats()
    assert st["n_delta_builds"] >= 8 and st["n_tombstones"] > 0
    assert (st["n_ext_rules"] > 0 and st["n_overlay_rules"] == 0) if ext else st["n_overlay_rules"] > 0, st
    c.reset_counters()
    got = c.classify_host(cols, count=True)
    _, slots = c.counters()
    want_cnt = np.zeros((max(1, len(slots)), 3), np.uint64)
    _cmp(got, emu.classify(c, cols, counters=want_cnt), cols)
    want_m = {int(slots[s]): tuple(int(x) for x in want_cnt[s]) for s in range(len(slots)) if slots[s] and want_cnt[s].any()}
    assert {k: tuple(v) for k, v in c.network_policy_metrics().items() if any(v)} == want_m


def emu_ip(v):
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def test_gpu_classification_concurrent_with_commits():
    """C5's shape, checked: a control thread applies Add/DeletePolicyRuleAddress ops and publishes
    a delta epoch per batch while the main thread queues classification launches on its own
    stream. Each launch is bound to one epoch (gpc_stream_epoch); its verdicts equal the emulation
    of that epoch's snapshot, and the final NetworkPolicyMetrics equal the per-launch emulated
    counters summed over the launches."""
    import torch
    wl = workload.config3(n_policies_per_dir=50, rules_per_policy=100)  # 10k rules
    n = 40000
    cols = workload.gen_packets(wl, n, seed=51)
    dev = torch.device("cuda", 0)
    signed = {4: np.int32, 2: np.int16, 1: np.uint8}  # device columns: the same bits in torch dtypes
    dcols = {k: torch.as_tensor(np.ascontiguousarray(v).view(signed[v.dtype.itemsize])).to(dev) for k, v in cols.items()}
    soa = gpc.pkt_soa_device(dcols)
    c = gpc.Classifier()
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    c.commit()
    snaps = {c.image_stats()["epoch"]: emu.snapshot(c)}
    stop, errors = threading.Event(), []
    rules = [r for r in wl.rules if r.get("from")]

    def control():
        rng = np.random.default_rng(52)
        added = []
        try:
            while not stop.is_set():
                for _ in range(25):
                    if added and rng.random() < 0.5:
                        rid, a, prio = added.pop(int(rng.integers(len(added))))
                        c.delete_policy_rule_address(rid, "src", [a], prio)
                    else:
                        r = rules[int(rng.integers(len(rules)))]
                        a = emu_ip(int(cols["src"][int(rng.integers(n))]))  # peers the batch does send from
                        c.add_policy_rule_address(r["flow_id"], "src", [a], r.get("priority"))
                        added.append((r["flow_id"], a, r.get("priority")))
                c.commit()
                snaps[c.image_stats()["epoch"]] = emu.snapshot(c)
                time.sleep(0.002)
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    s = torch.cuda.Stream(dev)
    c.reset_counters()
    th = threading.Thread(target=control, daemon=True)
    th.start()
    launches = []
    for i in range(48):
        out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
        c.classify_device(soa, n, out.data_ptr(), count=True, stream=s.cuda_stream)
        launches.append((c.stream_epoch(s.cuda_stream), out))
        time.sleep(0.004)
    stop.set()
    th.join()
    torch.cuda.synchronize(dev)
    assert not errors, errors
    epochs = sorted(set(e for e, _ in launches))
    assert len(epochs) >= 5, epochs  # the launches really did interleave with commits
    _, slots = c.counters()
    acc = np.zeros((max(1, len(slots)), 3), np.uint64)
    for e, out in launches:
        got = out.cpu().numpy().view(gpc.VERDICT_DTYPE).reshape(n, 2)
        _cmp(got, emu.classify_snapshot(snaps[e], cols, counters=acc), cols)
    want_m = {int(slots[i]): tuple(int(x) for x in acc[i]) for i in range(len(slots)) if slots[i] and acc[i].any()}
    assert {k: tuple(v) for k, v in c.network_policy_metrics().items() if any(v)} == want_m


def test_gpu_concurrent_commits_c3_vs_oracle():
    """C5 as it runs, at full scale: the C3 rule set (100k rules), a control thread
    replaying the seeded churn log of parity_C5.npz (address adds / deletes incl. base peers,
    uninstall / reinstall, priority reassignment) and publishing a delta epoch at every commit
    marker, while the main thread keeps launching classification on its own stream. For the first,
    a middle and the last commit, the control thread waits until a launch is bound to that epoch
    (gpc_stream_epoch); that launch's verdicts equal the C oracle over the ORACLE compiler's replay
    of the same op prefix (make_churn_fixture.py verdicts_at_k / verdicts). The background compactor
    is on: after the middle check the control thread keeps committing until a
    compacted base has been handed over, so the last checked epoch sits on a base the compactor
    built while launches were in flight, with the rest of the log in its catch-up journal."""
    import torch
    from oracle import parity
    from tests.golden import make_churn_fixture as mcf
    from tests.golden import make_parity_fixtures as fx
    f = mcf.load()
    wl, log, cols = mcf.inputs()
    assert mcf.log_digest(log) == str(f["log_sha256"]) and fx.cols_digest(cols) == str(f["cols_sha256"])
    n_commits = sum(1 for o in log if o["op"] == "commit")
    check = {k: f["at"][k] for k in f["at"]}
    check[n_commits] = f["verdicts"]
    assert len(check) == 3
    n = len(cols["src"])
    dev = torch.device("cuda", 0)
    signed = {4: np.int32, 2: np.int16, 1: np.uint8}
    dcols = {k: torch.as_tensor(np.ascontiguousarray(v).view(signed[v.dtype.itemsize])).to(dev) for k, v in cols.items()}
    soa = gpc.pkt_soa_device(dcols)
    c = gpc.Classifier(compact_after=256)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    c.commit()
    want_epoch = {}  # commit number -> epoch published for it (checked ones)
    bg_at = {}       # commit number -> background builds installed when it was checked
    mid = sorted(check)[1]
    waiting = {"epoch": None}
    seen = threading.Event()
    stop, errors = threading.Event(), []

    def control():
        k = [0]

        def on_commit():
            c.commit()
            k[0] += 1
            if k[0] in check:
                st = c.image_stats()
                e = st["epoch"]
                want_epoch[k[0]] = e
                bg_at[k[0]] = st["n_background_builds"]
                seen.clear()
                waiting["epoch"] = e
                if not seen.wait(120):
                    raise RuntimeError("no launch bound to epoch %d" % e)
            if k[0] == mid:  # let a compaction finish and hand over (empty commits install it)
                t0 = time.time()
                while c.image_stats()["n_background_builds"] <= bg_at[mid]:
                    if time.time() - t0 > 90:
                        raise RuntimeError("no background compaction handed over")
                    time.sleep(0.05)
                    c.commit()
            time.sleep(0.001)

        try:
            mcf.apply(c, log, on_commit)
        except Exception as e:  # surfaced in the main thread
            errors.append(e)
        finally:
            stop.set()

    s = torch.cuda.Stream(dev)
    th = threading.Thread(target=control, daemon=True)
    th.start()
    bound = {}  # epoch -> device verdicts of a launch bound to it
    while not stop.is_set() or waiting["epoch"] is not None:
        out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
        c.classify_device(soa, n, out.data_ptr(), stream=s.cuda_stream)
        e = c.stream_epoch(s.cuda_stream)
        if e == waiting["epoch"]:
            bound[e] = out
            waiting["epoch"] = None
            seen.set()
        if stop.is_set() and waiting["epoch"] is None:
            break
    th.join()
    torch.cuda.synchronize(dev)
    assert not errors, errors
    st = c.image_stats()
    assert st["n_delta_builds"] >= n_commits - 2, st  # the log went through delta epochs
    first, last = min(check), max(check)
    assert bg_at[last] > bg_at[first], (bg_at, st)  # a compacted base was handed over between them
    for k, want in sorted(check.items()):
        got = bound[want_epoch[k]].cpu().numpy().view(gpc.VERDICT_DTYPE).reshape(n, 2)[:len(want)]
        res = parity.compare(got, want)
        assert res["mismatches"] == 0, (k, res)


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_gpu_rccl_counter_allreduce_world1():
    """The path's only collective, on the device: the library's per-rule counters wrapped
    zero-copy (dist.device_counters) and all-reduced over an NCCL(=RCCL) group of world size 1
    (dist.all_reduce called directly); the reduced buffer maps to exactly gpc_metrics."""
    import torch
    import torch.distributed as tdist
    from antrea_amd import dist as gdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dev = torch.device("cuda", 0)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        wl = workload.config1(seed=61)
        cols = workload.gen_packets(wl, 50000, seed=61)
        c = gpc.Classifier()
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        c.commit()
        c.classify_host(cols, count=True)
        ptr, slots = c.counters()
        t = gdist.device_counters(ptr, len(slots), dev)
        before = t.clone()
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
        torch.cuda.synchronize(dev)
        assert torch.equal(t, before)
        got = {k: v for k, v in gdist.metrics_from_counters(t.cpu().numpy(), slots).items() if any(v)}
        assert got and got == {k: tuple(v) for k, v in c.network_policy_metrics().items() if any(v)}
    finally:
        tdist.destroy_process_group()


def test_gpu_replay_rebuilds_device_state():
    """gpc_replay (ReplayFlows for the device, client.go:1130-1152): every device buffer of the
    current epoch -- base image, journal pool (a delta epoch), IPv6 image -- is rebuilt from the
    host shadow state; verdicts are unchanged and counters restart from zero, as OVS's do when the
    agent replays its flows."""
    wl = workload.config1(seed=71)
    c = gpc.Classifier(ipv6=True)
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(workload.to_ipv6(wl, dual=True).rules))
    c.commit()
    c.add_policy_rule_address(wl.rules[0]["flow_id"], "src", ["10.10.0.77", "fd00:10::10.10.0.77"],
                              wl.rules[0].get("priority"))
    c.commit()
    st = c.image_stats()  # a delta epoch (IPv4: a point extension; IPv6: the journal): the pools must travel too
    assert st["n_ext_rules"] > 0 and st["v6_overlay_rules"] > 0, st
    cols = workload.gen_packets(wl, 20000, seed=71)
    v4 = c.classify_host(cols, count=True)
    v6 = c.classify6_host(workload.packets_to_v6(cols))
    m1 = {k: v for k, v in c.network_policy_metrics().items() if any(v)}
    e0 = c.image_stats()["epoch"]
    c.replay()
    assert c.image_stats()["epoch"] == e0 + 1
    assert not any(any(v) for v in c.network_policy_metrics().values())  # counters restart from zero
    assert (c.classify_host(cols, count=True) == v4).all()
    assert (c.classify6_host(workload.packets_to_v6(cols)) == v6).all()
    assert {k: v for k, v in c.network_policy_metrics().items() if any(v)} == m1
    c.add_policy_rule_address(wl.rules[1]["flow_id"], "src", ["10.10.0.78"], wl.rules[1].get("priority"))
    c.commit()  # delta commits continue on the replayed journal
    _cmp(c.classify_host(cols), emu.classify(c, cols), cols)
