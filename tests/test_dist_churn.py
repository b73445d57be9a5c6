"""Multi-rank churn on CPU (gloo, world size 2): every rank replicates one policy, so every rank
must apply ONE op stream (rule updates go to every GPU's epoch).

* test_replicated_op_log_world2: both ranks replay the same seeded op log (the C5 fixture's op
  mix -- address add/delete incl. original peers, uninstall / reinstall, ReassignFlowPriorities --
  over a small C3-shaped rule set) with a commit at each marker. Per commit the ranks must hold
  the same epoch contents: the same host base image, the same journal pool and header, the same
  full / delta build counts and the same realized flows. At the end both ranks' verdicts (host
  emulation of the kernel body) are identical and equal to the oracle classifier's.
* test_bench_churn_ops_world2: bench.py's C5 op stream (_ChurnOps, one seed on every rank) with a
  different commit batching per rank, then the catch-up of _churn_converge's first step: the
  realized flows and verdicts agree across ranks once both applied the same op prefix.
"""
import copy
import hashlib
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
N_PKTS = 400


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _small_c3():
    from antrea_amd import workload
    return workload.config3(seed=7, n_policies_per_dir=6, rules_per_policy=8)


def _epoch_digest(clf):
    """SHA-256 of what a commit publishes on the host side: base image, journal pool + header."""
    import ctypes as C
    h = hashlib.sha256()
    b, n, hdr, hb = clf.debug_image()
    if n:
        h.update(C.string_at(b, 4 * n))
        h.update(C.string_at(hdr, hb))
    p, pw, jh = clf.debug_epoch()
    if p and pw:
        h.update(C.string_at(p, 4 * pw))
    h.update(int(jh).to_bytes(4, "little"))
    st = clf.image_stats()
    h.update(repr((st["n_full_builds"], st["n_delta_builds"], st["n_overlay_rules"], st["n_tombstones"])).encode())
    return h.hexdigest()


def _log_worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from antrea_amd import gpc, workload
    from tests import emu
    from tests.golden import make_churn_fixture as mcf
    wl = _small_c3()
    log = mcf.ops(wl, seed=0xD15)[:900] + [{"op": "commit"}]
    clf = gpc.Classifier(compact_after=-1)  # synchronous: the epoch sequence is a function of the log alone
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    emu.commit_host(clf)
    digests = [_epoch_digest(clf)]

    def on_commit():
        emu.commit_host(clf)
        digests.append(_epoch_digest(clf))

    mcf.apply(clf, log, on_commit)
    cols = workload.gen_packets(wl, N_PKTS, seed=99)
    v = emu.classify(clf, cols)
    flows = sorted(clf.dump_flows())
    got = [None] * WORLD
    dist.all_gather_object(got, {"digests": digests, "flows": hashlib.sha256("\n".join(flows).encode()).hexdigest(),
                                 "verdicts": hashlib.sha256(v.tobytes()).hexdigest()})
    if rank == 0:
        np.save(os.path.join(outdir, "v.npy"), v)
        with open(os.path.join(outdir, "log.json"), "w") as f:
            import json
            json.dump({"ranks": got, "n_ops": len(log)}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_op_log_world2(tmp_path):
    import json
    from antrea_amd import gpc, workload
    from oracle import compiler as oc
    from oracle import ovs_cls
    from tests.golden import make_churn_fixture as mcf
    mp.start_processes(_log_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    with open(tmp_path / "log.json") as f:
        res = json.load(f)
    r0, r1 = res["ranks"]
    assert len(r0["digests"]) > 5 and r0["digests"] == r1["digests"]  # identical epochs, commit by commit
    assert len(set(r0["digests"])) > 5  # the epochs did change
    assert r0["flows"] == r1["flows"] and r0["verdicts"] == r1["verdicts"]
    # and the replicated verdicts are the oracle's
    wl = _small_c3()
    log = mcf.ops(wl, seed=0xD15)[:900]
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    mcf.apply(fnp, log)
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    pipe = ovs_cls.Pipeline(fnp.dump_flows(), tiers)
    cols = workload.gen_packets(wl, N_PKTS, seed=99)
    v = np.load(tmp_path / "v.npy")
    for i in range(N_PKTS):
        e, g = pipe.classify({k: int(c[i]) for k, c in cols.items()})
        for j, w in enumerate((e, g)):
            assert tuple(int(v[i, j][k]) for k in ("action", "conj_id", "table", "tier", "flags")) == \
                (w[0], w[1], w[2], w[3], w[4]), (i, j)


def _bench_worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import torch
    import bench
    from antrea_amd import gpc, workload
    from tests import emu
    wl = _small_c3()
    clf = gpc.Classifier(compact_after=-1)
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    emu.commit_host(clf)
    clf.commit = lambda: emu.commit_host(clf)  # no device here: host image + journal only
    ops = bench._ChurnOps(clf, wl, seed=1234)
    batch = (7, 31)[rank]  # rank-local batching, as the rate-driven control loops do
    for _ in range((1100 + 500 * rank) // batch):
        ops.apply(batch)
        clf.commit()
    t = torch.tensor([ops.issued], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ops.apply(int(t.item()) - ops.issued)
    clf.commit()
    v = emu.classify(clf, workload.gen_packets(wl, N_PKTS, seed=5))
    got = [None] * WORLD
    dist.all_gather_object(got, (ops.issued, hashlib.sha256("\n".join(sorted(clf.dump_flows())).encode()).hexdigest(),
                                 hashlib.sha256(v.tobytes()).hexdigest()))
    if rank == 0:
        with open(os.path.join(outdir, "bench.txt"), "w") as f:
            f.write(repr(got))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_churn_ops_world2(tmp_path):
    import ast
    mp.start_processes(_bench_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    got = ast.literal_eval((tmp_path / "bench.txt").read_text())
    assert got[0] == got[1], got
    assert got[0][0] >= 1500
