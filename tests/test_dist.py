"""Multi-rank path on CPU (gloo, world size 2): each rank commits the same rules, classifies its
own packet shard (host emulation of the kernel body, counters on) and the per-rule counters are
all-reduced with antrea_amd.dist -- the function bench.py applies to the device buffer over RCCL.
Rank 0 checks the reduced NetworkPolicyMetrics against the oracle classifier run over all shards,
including sessions (+new only for allow rules, network_policy.go:1917-1980)."""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
N_PER_RANK = 250


def _packets(wl, rank):
    from antrea_amd import workload
    cols = workload.gen_packets(wl, N_PER_RANK, seed=1000 + rank)
    rng = np.random.default_rng(77 + rank)
    u = rng.random(N_PER_RANK)
    # 70% +new+trk, 20% +trk only (-new: counted, no session), 10% +est+trk (skip flows -> BYPASS)
    cols["ct_state"] = np.where(u < 0.7, 0x21, np.where(u < 0.9, 0x20, 0x22)).astype(np.uint8)
    return cols


def _workload():
    from antrea_amd import workload
    return workload.config1(seed=21)


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from antrea_amd import dist as gdist
    from antrea_amd import gpc
    from tests import emu
    wl = _workload()
    clf = gpc.Classifier()
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    emu.commit_host(clf)
    _, slots = _slots(clf)
    cnt = np.zeros(gdist.COUNTER_WORDS * len(slots), dtype=np.uint64)
    v = emu.classify(clf, _packets(wl, rank), counters=cnt)
    np.save(os.path.join(outdir, "v%d.npy" % rank), v)
    t = torch.from_numpy(cnt.view(np.int64).copy())
    gdist.allreduce_counters(t)
    if rank == 0:
        np.save(os.path.join(outdir, "reduced.npy"), t.numpy().view(np.uint64))
        np.save(os.path.join(outdir, "slots.npy"), np.asarray(slots, dtype=np.uint32))
    dist.barrier()
    dist.destroy_process_group()


def _slots(clf):
    """slot -> conj map of the committed image without touching a device (gpc_counters returns it
    together with the (null on CPU) device pointer)."""
    import ctypes as C
    from antrea_amd import gpc
    p = C.POINTER(C.c_uint64)()
    s = C.POINTER(C.c_uint32)()
    n = C.c_size_t()
    rc = clf.lib.gpc_counters(clf.h, C.byref(p), C.byref(s), C.byref(n))
    assert rc == 0
    return None, [s[i] for i in range(n.value)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_counter_allreduce_world2(tmp_path):
    from antrea_amd import dist as gdist
    from oracle import compiler as oc
    from oracle import ovs_cls
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    reduced = np.load(tmp_path / "reduced.npy")
    slots = np.load(tmp_path / "slots.npy").tolist()
    got = gdist.metrics_from_counters(reduced, slots)
    wl = _workload()
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), tiers)
    for rank in range(WORLD):
        cols = _packets(wl, rank)
        v = np.load(tmp_path / ("v%d.npy" % rank))
        for i in range(N_PER_RANK):
            e, g = pipe.classify({k: int(c[i]) for k, c in cols.items()})
            assert (int(v[i, 0]["action"]), int(v[i, 0]["conj_id"])) == (e[0], e[1]), (rank, i)
            assert (int(v[i, 1]["action"]), int(v[i, 1]["conj_id"])) == (g[0], g[1]), (rank, i)
    d = pipe.metric_dumps()
    want = oc.network_policy_metrics(d["EgressMetric"], d["IngressMetric"])
    want = {k: tuple(v) for k, v in want.items() if any(v)}
    got = {k: v for k, v in got.items() if any(v)}
    assert got == want
    assert any(p != s for p, _, s in got.values())  # some -new packets: sessions < packets


def test_shard_range_covers():
    from antrea_amd import dist as gdist
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rs = [gdist.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
