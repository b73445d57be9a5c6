"""Generates tests/golden/parity_C5.npz: the C oracle's verdicts and metrics for C3 after a seeded
control-plane op log -- config 5's churn path (TEST INFRASTRUCTURE; run here on the CPU).

    python tests/golden/make_churn_fixture.py

The op log (`ops`, deterministic from the workload and SEED) mixes the reference's churn entry
points:
  * AddPolicyRuleAddress / DeletePolicyRuleAddress (network_policy.go:1661-1710) on both address
    sides: new /32 peers and new ofports added, added ones and ORIGINAL ones deleted (the base
    image's flows then need tombstones), a clause emptied now and then;
  * UninstallPolicyRuleFlows (:1570) of whole rules, half of them reinstalled later
    (InstallPolicyRuleFlows :1160);
  * ReassignFlowPriorities (:1873) of single rules to free priorities of their table;
  * a "commit" marker every COMMIT_EVERY ops (the product publishes a delta epoch there; the
    oracle has no epochs).
The ORACLE compiler replays the log over the C3 rule set; its final flow dump is loaded into the C
OVS classifier, which classifies N seeded packets with counters on. Stored: verdicts, metrics and
SHA-256 digests of the rules, the op log and the packets (drift is detected, never compared).
"""
from __future__ import annotations

import copy
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from antrea_amd import workload  # noqa: E402
from oracle import parity  # noqa: E402
from tests.golden import make_parity_fixtures as fx  # noqa: E402

SEED = 0xC5C5
N_ADDR_OPS = 3000
N_UNINSTALL = 200
N_REASSIGN = 30
COMMIT_EVERY = 100
N_PKTS, PKT_SEED = 100_000, 0xF1C6
PATH = os.path.join(HERE, "parity_C5.npz")
# intermediate states checked by the concurrent-commit device test (tests/test_gpu_boundary.py):
# the oracle's verdicts for the first N_AT packets after commit marker k of the log (1-based; the
# final state is `verdicts`)
AT_COMMITS = (1, 17)
N_AT = 20_000


def _ip(v):
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def ops(wl, seed=SEED):
    """The op log over wl.rules (a list of dicts; the rule dicts of reinstalls are copies)."""
    rng = np.random.default_rng(seed)
    rules = {r["flow_id"]: r for r in wl.rules}
    live = set(rules)
    addrs = {fid: {"src": list(r.get("from") or []), "dst": list(r.get("to") or [])} for fid, r in rules.items()}
    prio = {fid: r.get("priority") for fid, r in rules.items()}
    used = {}
    for r in wl.rules:
        if r.get("priority") is not None:
            used.setdefault(r["table"], set()).add(r["priority"])
    uninstalled = []
    kinds = (["addr"] * N_ADDR_OPS) + (["uninstall"] * N_UNINSTALL) + (["reassign"] * N_REASSIGN)
    kinds += ["reinstall"] * (N_UNINSTALL // 2)
    order = rng.permutation(len(kinds))
    log = []
    fids = sorted(rules)
    for j, k in enumerate(order):
        kind = kinds[k]
        if kind == "reinstall":
            if not uninstalled:
                kind = "addr"
            else:
                fid = uninstalled.pop(int(rng.integers(len(uninstalled))))
                r = copy.deepcopy(rules[fid])
                r["from"], r["to"] = copy.deepcopy(addrs[fid]["src"]), copy.deepcopy(addrs[fid]["dst"])
                if prio[fid] is not None:
                    r["priority"] = prio[fid]
                log.append({"op": "install", "rule": r})
                live.add(fid)
        if kind == "uninstall":
            fid = fids[int(rng.integers(len(fids)))]
            if fid not in live:
                kind = "addr"
            else:
                log.append({"op": "uninstall", "fid": fid})
                live.discard(fid)
                uninstalled.append(fid)
        if kind == "reassign":
            fid = fids[int(rng.integers(len(fids)))]
            r = rules[fid]
            if fid not in live or prio[fid] is None:
                kind = "addr"
            else:
                t = r["table"]
                while True:
                    p = int(rng.integers(100, 65001))
                    if p not in used[t]:
                        break
                used[t].discard(prio[fid])
                used[t].add(p)
                log.append({"op": "reassign", "table": t, "from": prio[fid], "to": p})
                prio[fid] = p
        if kind == "addr":
            fid = fids[int(rng.integers(len(fids)))]
            if fid not in live:
                continue
            side = "src" if rng.random() < 0.5 else "dst"
            cur = addrs[fid][side]
            if not cur:
                side = "dst" if side == "src" else "src"
                cur = addrs[fid][side]
                if not cur:
                    continue
            if rng.random() < 0.55 or len(cur) == 1 and rng.random() < 0.8:
                proto = cur[0]
                if isinstance(proto, dict) and "ofport" in proto:
                    a = {"ofport": int(rng.integers(1, 400))}
                else:
                    a = _ip(int(rng.integers(0, 1 << 32)))
                if a in cur:
                    continue
                cur.append(a)
                log.append({"op": "add", "fid": fid, "side": side, "addrs": [a], "priority": prio[fid]})
            else:
                a = cur.pop(int(rng.integers(len(cur))))
                log.append({"op": "del", "fid": fid, "side": side, "addrs": [a], "priority": prio[fid]})
        if (j + 1) % COMMIT_EVERY == 0:
            log.append({"op": "commit"})
    log.append({"op": "commit"})
    return log


def apply(client, log, on_commit=None):
    """Replays the op log through an openflow.Client NP surface (oracle compiler or product)."""
    for o in log:
        k = o["op"]
        if k == "add":
            client.add_policy_rule_address(o["fid"], o["side"], o["addrs"], o["priority"])
        elif k == "del":
            client.delete_policy_rule_address(o["fid"], o["side"], o["addrs"], o["priority"])
        elif k == "uninstall":
            client.uninstall_policy_rule_flows(o["fid"])
        elif k == "install":
            client.install_policy_rule_flows(copy.deepcopy(o["rule"]))
        elif k == "reassign":
            client.reassign_flow_priorities({o["from"]: o["to"]}, o["table"])
        elif k == "commit" and on_commit is not None:
            on_commit()


def log_digest(log) -> str:
    return hashlib.sha256(json.dumps(log, sort_keys=True).encode()).hexdigest()


def inputs():
    wl = workload.config3()
    log = ops(wl)
    cols = workload.gen_packets(wl, N_PKTS, seed=PKT_SEED)
    return wl, log, cols


def make():
    from oracle import compiler as oc
    from oracle.cls_c import CPipeline
    t0 = time.time()
    wl, log, cols = inputs()
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    t1 = time.time()
    at = {}
    n_commit = [0]

    def on_commit():
        n_commit[0] += 1
        if n_commit[0] in AT_COMMITS:
            p = CPipeline(fnp.dump_flows(), parity.tiers_of(wl))
            sub = {k: v[:N_AT] for k, v in cols.items()}
            at[n_commit[0]] = np.ascontiguousarray(p.classify(sub, threads=parity.cpu_threads())).view(np.uint32).reshape(-1, 4)

    apply(fnp, log, on_commit)
    t2 = time.time()
    pipe = CPipeline(fnp.dump_flows(), parity.tiers_of(wl))
    want = pipe.classify(cols, threads=parity.cpu_threads(), count=True)
    t3 = time.time()
    m = parity.oracle_metrics(pipe)
    conj = np.array(sorted(m), np.uint32)
    met = np.array([m[int(c)] for c in conj], np.uint64).reshape(-1, 3)
    counts = {k: sum(1 for o in log if o["op"] == k) for k in ("add", "del", "uninstall", "install", "reassign", "commit")}
    np.savez_compressed(PATH, verdicts=np.ascontiguousarray(want).view(np.uint32).reshape(-1, 4), metric_conj=conj,
                        metric_val=met, cols_sha256=fx.cols_digest(cols), rules_sha256=fx.rules_digest(wl),
                        log_sha256=log_digest(log), n_flows=pipe.n_flows, op_counts=json.dumps(counts),
                        at_commits=np.array(sorted(at), np.int32),
                        **{"verdicts_at_%d" % k: v for k, v in at.items()})
    print("C5 fixture: %s, %d flows after the log; compile %.0f s, log %.0f s, classify %.1f s"
          % (counts, pipe.n_flows, t1 - t0, t2 - t1, t3 - t2))


def load() -> dict:
    with np.load(PATH, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["verdicts"] = np.ascontiguousarray(d["verdicts"]).view(parity.VERDICT_NP).reshape(-1, 2)
    d["at"] = {int(k): np.ascontiguousarray(d["verdicts_at_%d" % k]).view(parity.VERDICT_NP).reshape(-1, 2)
               for k in d.get("at_commits", [])}
    d["metrics"] = {int(c): tuple(int(x) for x in v) for c, v in zip(d["metric_conj"], d["metric_val"])}
    return d


if __name__ == "__main__":
    make()
