"""GPU: the cost of a C5 churn state, frozen. Builds C3, then moves it through churn states without
the concurrent control thread (no compactor: compact_after = -1), timing 10 launches of the 64 M
packet batch in each state. Separates the extension probe, the journal walk and the launch shape
(grouping, split stages) from commit interference -- bench.py C5 times them all together.

    python tools/c5_state.py [--ext-ops 100000] [--journal-ops 300] [--group 0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ext-ops", type=int, default=100000)
    ap.add_argument("--journal-ops", type=int, default=300)
    ap.add_argument("--group", type=int, default=0)
    ap.add_argument("--packets", type=int, default=1 << 26)
    args = ap.parse_args()
    import torch
    import bench
    from antrea_amd import gpc, workload
    dp = (bench._HostEmuPath if os.environ.get("GPC_BENCH_HOST_EMU") else bench._HipPath)(0)
    wl = workload.config3()
    clf = gpc.Classifier(device=0, group_packets=args.group, compact_after=-1)
    dp.bind(clf, False)
    clf.initialize()
    clf.batch_install_policy_rule_flows(wl.rules)
    dp.commit()
    n = args.packets
    cols = workload.gen_packets_torch(wl, n, seed=workload.PKT_SEED, device=dp.dev)
    out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dp.dev)
    soa = gpc.pkt_soa_device(cols)
    stream = dp.stream(own=False)
    k_c = 8192
    idx = (torch.arange(k_c, dtype=torch.int64) * min(n, 1 << 20)) // k_c
    cands = bench.churn_candidates(wl, bench._host_sample(cols, idx.to(dp.dev)))
    res = []

    def measure(label):
        for _ in range(2):
            dp.classify(soa, n, out, True, stream)
        dp.sync()
        dp.set_launch_timing(10)
        ev = [dp.event() for _ in range(2)]
        ev[0].record(stream)
        for _ in range(10):
            dp.classify(soa, n, out, True, stream)
        ev[1].record(stream)
        dp.sync()
        lt = dp.launch_times()
        dp.set_launch_timing(0)
        st = clf.image_stats()
        r = {"state": label, "ms_per_step": round(ev[0].elapsed_time(ev[1]) / 10, 3),
             "kernels": {k: round(v["total_ms"] / max(1, v["launches"]), 3) for k, v in lt.items()},
             "journal_rules": st["n_overlay_rules"], "tombstones": st["n_tombstones"],
             "ext_rules": st["n_ext_rules"], "ext_values": st["n_ext_values"], "pool_MB": round(st["overlay_bytes"] / 1e6, 1)}
        print(json.dumps(r), flush=True)
        res.append(r)

    def churn(ops, k):
        t = time.time()
        done = 0
        while done < k:
            m = min(126, k - done)
            ops.apply(m)
            dp.commit()
            done += m
            if time.time() - t > 20:
                print("[c5_state] %d / %d ops" % (done, k), file=sys.stderr, flush=True)
                t = time.time()

    measure("base")
    ext_only = {"del_base": 0.0, "readd_base": 0.0, "uninstall": 0.0, "reinstall": 0.0, "reassign": 0.0}
    ops = bench._ChurnOps(clf, wl, seed=1234, mix="mixed", cands=cands, weights=ext_only)
    churn(ops, args.ext_ops)
    measure("extensions (%d add/delete ops)" % args.ext_ops)
    jops = bench._ChurnOps(clf, wl, seed=99, mix="mixed", cands=[],
                           weights={"add_hit": 0.0, "del_add": 0.0, "del_base": 0.45, "readd_base": 0.45,
                                    "uninstall": 0.04, "reinstall": 0.03, "reassign": 0.03})
    jops.cur = ops.cur  # (the same live rule state)
    jops.prio, jops.used, jops.live = ops.prio, ops.used, ops.live
    for step in range(3):
        churn(jops, args.journal_ops)
        measure("+ journal (%d ops)" % ((step + 1) * args.journal_ops))
    print(json.dumps({"c5_state": res}))


if __name__ == "__main__":
    main()
