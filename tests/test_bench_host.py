"""Host-side pieces of bench.py that run without a GPU (C5 control loop)."""
import threading
import time

import numpy as np
import pytest

import bench
from antrea_amd import workload


class _Stub:
    def __init__(self):
        self.ops = 0
        self.commits = 0

    def add_policy_rule_address(self, *a):
        self.ops += 1

    def delete_policy_rule_address(self, *a):
        self.ops += 1

    def uninstall_policy_rule_flows(self, *a):
        self.ops += 1

    def install_policy_rule_flows(self, *a):
        self.ops += 1

    def reassign_flow_priorities(self, *a):
        self.ops += 1

    def commit(self):
        self.commits += 1
        time.sleep(0.002)


def test_churn_loop_paces_ops_and_records_latency():
    wl = workload.config1()
    stub, rec, stop = _Stub(), [], threading.Event()
    ops = bench._ChurnOps(stub, wl, seed=1, mix="uniform")
    th = threading.Thread(target=bench._churn_loop, args=(ops, 5000.0, 2000, stop, rec))
    th.start()
    time.sleep(0.5)
    stop.set()
    th.join()
    n = sum(r[0] for r in rec)
    assert n == stub.ops == ops.issued and len(rec) == stub.commits
    ops = n
    assert 1500 <= ops <= 3500  # ~5000 ops/s for 0.5 s
    assert all(len(r[2]) == r[0] and (r[2] >= 0).all() for r in rec)


@pytest.mark.parametrize("mix", ["mixed", "uniform"])
def test_churn_ops_same_seed_same_stream(mix):
    """C5 at N>1: every rank draws the same op sequence, whatever its batching."""
    wl = workload.config3(seed=5, n_policies_per_dir=6, rules_per_policy=10) if mix == "mixed" else workload.config1()
    cands = bench.churn_candidates(wl, workload.gen_packets(wl, 2000, seed=3)) if mix == "mixed" else None

    class Rec(_Stub):
        def __init__(self):
            super().__init__()
            self.seq = []

        def add_policy_rule_address(self, *a):
            self.seq.append(("add",) + tuple(map(str, a)))

        def delete_policy_rule_address(self, *a):
            self.seq.append(("del",) + tuple(map(str, a)))

        def uninstall_policy_rule_flows(self, *a):
            self.seq.append(("uninstall",) + tuple(map(str, a)))

        def install_policy_rule_flows(self, r):
            self.seq.append(("install", r["flow_id"], str(r["from"]), str(r["to"]), r.get("priority")))

        def reassign_flow_priorities(self, *a):
            self.seq.append(("reassign",) + tuple(map(str, a)))

    a, b = Rec(), Rec()
    w = {"uninstall": 0.03, "reinstall": 0.02, "reassign": 0.03}
    oa = bench._ChurnOps(a, wl, seed=1234, mix=mix, cands=cands, weights=w)
    ob = bench._ChurnOps(b, wl, seed=1234, mix=mix, cands=cands, weights=w)
    for _ in range(50):
        oa.apply(7)
    for _ in range(7):
        ob.apply(50)
    assert a.seq == b.seq[:350] and len(a.seq) == 350


def test_grouping_label_from_launches():
    """The bench line's packet_grouping field names what ran (no GPU: launch names only)."""
    import bench
    from antrea_amd import gpc
    st = {"group_key": gpc.GROUP_KEY_ADDR}
    assert bench._grouping_label(st, {"classify_egress": {}}, False) == "off"
    lab = bench._grouping_label(st, {"group_tiles": {}, "unpermute": {}}, False)
    assert lab.startswith("key: top 8 bits of nw_src") and lab.endswith("results un-permuted")
    assert "IPv6 code columns" in bench._grouping_label(st, {"group_tiles": {}}, True)
    assert "scan-length" in bench._grouping_label({"group_key": gpc.GROUP_KEY_SCAN}, {"group_tiles": {}}, False)


def _rank_launch_worker(rank, port, outdir):
    import json
    import os

    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    # the classify call is stubbed: what gpc_launch_times would report for this rank's timed region
    launches = {"classify_egress": {"mean_ms": 3.0 + rank, "launches": 10},
                "classify_ingress": {"mean_ms": 4.5 + rank, "launches": 10}}
    if rank == 1:
        launches["group_tiles"] = {"mean_ms": 0.7, "launches": 10}
    got = bench._gather_rank_launch_ms(launches, torch.device("cpu"), 2)
    with open(os.path.join(outdir, "r%d.json" % rank), "w") as f:
        json.dump(got, f)
    dist.destroy_process_group()


def test_rank_launch_times_world2(tmp_path):
    """N > 1 line assembly: every rank's per-launch HIP-event times reach rank 0
    in rank order, launch kinds a rank did not run are absent from its entry."""
    import json
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank_launch_worker, args=(port, str(tmp_path)), nprocs=2, join=True)
    for r in (0, 1):
        got = json.load(open(tmp_path / ("r%d.json" % r)))
        assert got == [{"classify_egress": 3.0, "classify_ingress": 4.5},
                       {"group_tiles": 0.7, "classify_egress": 4.0, "classify_ingress": 5.5}]


@pytest.mark.parametrize("mix", ["mixed", "uniform"])
def test_churn_op_log_replays_on_the_oracle(mix):
    """C5 parity: the op log bench._ChurnOps records, replayed on the
    oracle compiler, gives the flows the product compiler realized applying the same ops -- for the
    mixed stream every kind of op (adds of peers the batch sends, deletes of adds and of base
    ipBlock peers, re-adds, uninstall / reinstall, priority reassignment) occurs."""
    import copy

    from antrea_amd import gpc
    from oracle import compiler as oc
    from oracle.parity import replay_churn
    wl = workload.config3(seed=5, n_policies_per_dir=6, rules_per_policy=10)
    clf = gpc.Classifier(compact_after=-1)
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    cands = bench.churn_candidates(wl, workload.gen_packets(wl, 4000, seed=3)) if mix == "mixed" else None
    w = {"uninstall": 0.03, "reinstall": 0.02, "reassign": 0.03} if mix == "mixed" else None
    ops = bench._ChurnOps(clf, wl, seed=99, mix=mix, cands=cands, base_frac=0.2, weights=w)
    for _ in range(40):
        ops.apply(5)
    assert len(ops.log) == 200
    if mix == "mixed":
        assert len(cands) > 20
        assert all(ops.counts[k] > 0 for k in ops.kinds), ops.counts
        assert {o["op"] for o in ops.log} == {"add", "del", "uninstall", "install", "reassign"}
    else:
        assert {o["op"] for o in ops.log} == {"add", "del"}
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    assert replay_churn(fnp, ops.log) == 200
    assert sorted(fnp.dump_flows()) == sorted(clf.dump_flows())


def test_churn_candidates_complete_rules():
    """Every candidate add of the mixed C5 stream makes its rule complete for the packet it came
    from: after adding it, the emulated verdict of that packet is decided by that rule or by a rule
    ranked above it (never NO_MATCH in the rule's stage)."""
    import copy

    from antrea_amd import gpc
    from tests import emu
    wl = workload.config3(seed=5, n_policies_per_dir=6, rules_per_policy=10)
    cols = workload.gen_packets(wl, 3000, seed=3)
    cands = bench.churn_candidates(wl, cols)
    assert cands
    side, fid, v = cands[0]
    clf = gpc.Classifier(compact_after=-1)
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    rule = next(r for r in wl.rules if r["flow_id"] == fid)
    clf.rule_addr_ip4(True, fid, side, v, rule.get("priority"))
    emu.commit_host(clf)
    key = "src" if side == "src" else "dst"
    i = int(np.nonzero(cols[key] == np.uint32(v))[0][0])
    one = {k: a[i:i + 1] for k, a in cols.items()}
    got = emu.classify(clf, one)[0, 0 if side == "dst" else 1]
    assert got["action"] != 1 and got["conj_id"] != 0


def _run_bench(args, env_extra, timeout=600):
    import json
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, cwd=root,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(line[-1]) if line else None), p.stderr


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself
    (RANK / WORLD_SIZE / MASTER_* set by bench.py), they rendezvous (gloo here: the classify call
    is the host emulation of the committed image, GPC_BENCH_HOST_EMU), all-reduce the per-rule
    counters, gather every rank's launch times, and rank 0 prints the one line with n_gpus == 2
    and its parity stamp against the oracle."""
    rc, res, err = _run_bench(["--gpus", "2", "--config", "C1", "--packets", "4096", "--steps", "3", "--warmup", "1"],
                              {"GPC_BENCH_HOST_EMU": "1"})
    assert rc == 0, err[-3000:]
    assert res["n_gpus"] == 2 and res["config"]["parallelism"].endswith("x2, rules replicated")
    assert res["data"].startswith("host-emulation")
    per_rank = res["kernel_ms_by_launch_per_rank"]
    assert len(per_rank) == 2 and all("classify_both" in r for r in per_rank)
    assert res["parity"]["checked"] == 4096 and res["parity"]["mismatches"] == 0
    assert "rank 0's shard of 2" in res["parity"]["sample"]
    assert res["counters_allreduced"]["slots"] > 0 and res["counters_allreduced"]["packets"] > 0
    assert res["value"] > 0 and res["steps"] == 3


def test_bench_gpus_mismatch_with_launcher_fails():
    """--gpus that disagrees with the launcher's WORLD_SIZE is an error, not a silent 1-GPU line."""
    rc, res, err = _run_bench(["--gpus", "4", "--config", "C1", "--packets", "1024"],
                              {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "GPC_BENCH_HOST_EMU": "1"}, timeout=120)
    assert rc == 2 and res is None and "WORLD_SIZE=2" in err
