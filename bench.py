"""Headline benchmark: Mpps classified (5-tuple -> rule verdict, both policy stages) @100k rules.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--packets 67108864]
    python bench.py --config C5   # C3 + AddPolicyRuleAddress/DeletePolicyRuleAddress churn

C5 (BASELINE config 5): the C3 rule set with address updates interleaved with
classification. A control thread applies `--churn-rate` ops/s (alternating add / delete of /32
peers on random rules; every op due so far is applied and published with one gpc_commit, i.e. one
delta epoch) while the timed classification loop runs on its own stream; the line adds the update
latency (op due -> commit returned) percentiles next to the Mpps measured under churn.

One process per GPU (torchrun for N > 1). Each rank builds the same rule set (C3 = 100k rules),
classifies its own packet shard (weak scaling: `--packets` per GPU, inputs resident in HBM before
the timed region) and, when counters are on, all-reduces the per-rule counters over RCCL at the
end of the run (the only collective of the path). A step = one gpc_classify call
over the whole per-GPU batch (two kernel launches without Services: egress stage, ingress stage).

Rank 0 at N = 1 also (all after the timed region, none of it timed):
  * parity: a 64k-packet strided sample of the timed batch and its device verdicts are checked
    packet for packet against the C oracle (oracle/ovs_cls.c over the ORACLE compiler's flows),
    which a spawned CPU process prepares while the GPU works -> "parity": {checked, mismatches};
  * cpu_baseline: the same C oracle timed on the host cores (bounded sample, see oracle/parity.py);
  * roofline: the dominant kernel's measured L2<->fabric bytes per launch (rocprofv3 FETCH_SIZE x2 +
    WRITE_SIZE, separate child passes, MI355X_MICROARCH.md HBM section) / its mean duration from HIP
    events recorded around every launch of the timed region (gpc_launch_times), against 8 TB/s; the
    whole step's figures and every launch kind's beside it.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
PARITY_SAMPLE = 1 << 16
# rocprofv3 passes (one run each: FETCH_SIZE takes 3 of the 4 TCC counter slots)
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"),
              # what bounds a gather kernel below the bandwidth roof: wave-parked (s_waitcnt) share
              # of wave cycles, vector-memory / scalar / vector instructions per wave
              ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU",
               "SQ_INSTS_VALU"))


def _log(msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    print("[bench %.0fs] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


_T0 = time.time()


def _lbar(wl, clf, n=20000, family=4):
    """Mean distinct 64-B image lines one packet's evaluation reads (instrumented host emulation of
    the same image, tests/csrc/emu.cpp), i.e. L-bar of SURVEY §8(d) -- a diagnostic of the
    algorithm, not a measured byte count."""
    try:
        from tests import emu
        from antrea_amd import workload
        cols = workload.gen_packets(wl, n, seed=12345)
        emu.stats(reset=True)
        if family == 6:
            emu.classify6(clf, workload.packets_to_v6(cols))
        else:
            emu.classify(clf, cols)
        s = emu.stats()
        return s[6] / max(1, s[7])
    except Exception as e:  # pragma: no cover - g++ missing
        print("L-bar unavailable: %s" % e, file=sys.stderr)
        return None


class _ChurnOps:
    """The C5 op stream, drawn from one seeded generator. Every rank uses the same seed and the same
    candidate list, so all ranks apply one op stream (they replicate one policy); only how the ops
    are batched into commits is rank-local. `log` records every op in the order applied, as dicts
    the oracle replays (oracle/parity.py replay_churn).

    mix "uniform" (round 5): alternating add / delete of uniformly random /32 source peers on random
    rules -- packets almost never hit them. mix "mixed" (default): the reference's churn entry points
    at rates that move traffic (`MIX`, per op):
      * AddPolicyRuleAddress of a /32 the timed batch sends (`cands`: for a sampled packet, a rule
        whose other clauses it matches, so the rule completes for it: ingress rules get the source
        in From, egress rules the destination in To) and DeletePolicyRuleAddress of earlier adds
        (network_policy.go:1661-1710; point extensions of the base records);
      * DeletePolicyRuleAddress of a rule's own ipBlock peer (the base record is tombstoned and the
        rule journaled) and the later re-add of such a peer;
      * UninstallPolicyRuleFlows (:1570) of whole rules and InstallPolicyRuleFlows (:1160) of some
        of them again;
      * ReassignFlowPriorities (:1873) of one rule to a free priority of its table."""

    MIX = (("add_hit", 0.45), ("del_add", 0.35), ("del_base", 0.09), ("readd_base", 0.10), ("uninstall", 0.0012),
           ("reinstall", 0.0008), ("reassign", 0.0010))
    # (the del_base / readd_base share is scaled by `base_frac` / 0.19: --churn-base-frac)

    def __init__(self, clf, wl, seed, mix="mixed", cands=None, base_frac=0.005, weights=None):
        import numpy as np
        self.clf = clf
        self.rng = np.random.default_rng(seed)
        self.mix = mix
        self.rules = [r for r in wl.rules if r.get("from")]
        self.added = []
        self.issued = 0
        self.log = []
        self.fast = getattr(clf, "rule_addr_ip4", None)  # the library's per-op cost, not string marshalling
        if mix == "uniform":
            return
        import copy
        self.by_fid = {r["flow_id"]: r for r in wl.rules}
        self.fids = sorted(self.by_fid)
        self.live = set(self.fids)
        self.prio = {f: r.get("priority") for f, r in self.by_fid.items()}
        self.cur = {f: {"src": copy.copy(r.get("from") or []), "dst": copy.copy(r.get("to") or [])}
                    for f, r in self.by_fid.items()}
        self.used = {}
        for r in wl.rules:
            if r.get("priority") is not None:
                self.used.setdefault(r["table"], set()).add(r["priority"])
        self.cands = cands if cands is not None else []
        self.added_set = set()
        self.base_gone = []  # (fid, side, addr) deleted base peers, re-addable
        self.uninstalled = []
        w = dict(self.MIX)
        sc = base_frac / (w["del_base"] + w["readd_base"])
        w["del_base"] *= sc
        w["readd_base"] *= sc
        w.update(weights or {})
        self.kinds = list(w)
        self.cum = np.cumsum([w[k] for k in self.kinds])
        self.cum /= self.cum[-1]
        self.counts = {k: 0 for k in self.kinds}

    # --- ops (each records itself; returns False when not applicable now)
    def _addr(self, add, fid, side, v):
        a = _ip4(v)
        if self.fast:
            self.fast(add, fid, side, v, self.prio[fid])
        elif add:
            self.clf.add_policy_rule_address(fid, side, [a], self.prio[fid])
        else:
            self.clf.delete_policy_rule_address(fid, side, [a], self.prio[fid])
        self.log.append({"op": "add" if add else "del", "fid": fid, "side": side, "addrs": [a],
                         "priority": self.prio[fid]})

    def _add_hit(self):
        rng = self.rng
        for _ in range(8):
            if not len(self.cands):
                return False
            side, fid, v = self.cands[int(rng.integers(len(self.cands)))]
            key = (fid, side, v)
            if fid not in self.live or key in self.added_set:
                continue
            self._addr(True, fid, side, v)
            self.added_set.add(key)
            self.added.append(key)
            self.cur[fid][side].append(_ip4(v))
            return True
        return False

    def _del_add(self):
        rng = self.rng
        for _ in range(8):
            if not self.added:
                return False
            j = int(rng.integers(len(self.added)))
            fid, side, v = self.added[j]
            if fid not in self.live:
                continue
            self.added[j] = self.added[-1]
            self.added.pop()
            self.added_set.discard((fid, side, v))
            self._addr(False, fid, side, v)
            self.cur[fid][side].remove(_ip4(v))
            return True
        return False

    def _del_base(self):
        rng = self.rng
        for _ in range(8):
            fid = self.fids[int(rng.integers(len(self.fids)))]
            if fid not in self.live:
                continue
            r = self.by_fid[fid]
            side = "src" if r["direction"] == "In" else "dst"  # the ipBlock side
            base = [a for a in self.cur[fid][side] if isinstance(a, dict)]
            if not base:
                continue
            a = base[int(rng.integers(len(base)))]
            self.clf.delete_policy_rule_address(fid, side, [a], self.prio[fid])
            self.log.append({"op": "del", "fid": fid, "side": side, "addrs": [a], "priority": self.prio[fid]})
            self.cur[fid][side].remove(a)
            self.base_gone.append((fid, side, a))
            return True
        return False

    def _readd_base(self):
        rng = self.rng
        for _ in range(8):
            if not self.base_gone:
                return False
            j = int(rng.integers(len(self.base_gone)))
            fid, side, a = self.base_gone[j]
            if fid not in self.live:
                continue
            self.base_gone[j] = self.base_gone[-1]
            self.base_gone.pop()
            self.clf.add_policy_rule_address(fid, side, [a], self.prio[fid])
            self.log.append({"op": "add", "fid": fid, "side": side, "addrs": [a], "priority": self.prio[fid]})
            self.cur[fid][side].append(a)
            return True
        return False

    def _uninstall(self):
        fid = self.fids[int(self.rng.integers(len(self.fids)))]
        if fid not in self.live:
            return False
        self.clf.uninstall_policy_rule_flows(fid)
        self.log.append({"op": "uninstall", "fid": fid})
        self.live.discard(fid)
        self.uninstalled.append(fid)
        return True

    def _reinstall(self):
        import copy
        if not self.uninstalled:
            return False
        fid = self.uninstalled.pop(int(self.rng.integers(len(self.uninstalled))))
        r = dict(self.by_fid[fid])
        r["from"], r["to"] = copy.copy(self.cur[fid]["src"]), copy.copy(self.cur[fid]["dst"])
        if self.prio[fid] is not None:
            r["priority"] = self.prio[fid]
        self.clf.install_policy_rule_flows(r)
        self.log.append({"op": "install", "rule": r})
        self.live.add(fid)
        return True

    def _reassign(self):
        rng = self.rng
        fid = self.fids[int(rng.integers(len(self.fids)))]
        if fid not in self.live or self.prio[fid] is None:
            return False
        t = self.by_fid[fid]["table"]
        while True:
            p = int(rng.integers(100, 65001))
            if p not in self.used[t]:
                break
        self.clf.reassign_flow_priorities({self.prio[fid]: p}, t)
        self.log.append({"op": "reassign", "table": t, "from": self.prio[fid], "to": p})
        self.used[t].discard(self.prio[fid])
        self.used[t].add(p)
        self.prio[fid] = p
        return True

    def apply(self, k):
        if self.mix == "uniform":
            return self._apply_uniform(k)
        import numpy as np
        rng = self.rng
        for _ in range(k):
            kind = self.kinds[int(np.searchsorted(self.cum, rng.random(), side="right"))]
            if not getattr(self, "_" + kind)():
                kind = "add_hit"
                if not self._add_hit():
                    kind = "del_add"
                    self._del_add()
            self.counts[kind] += 1
        self.issued += k

    def _apply_uniform(self, k):
        rng, clf, fast = self.rng, self.clf, self.fast
        for _ in range(k):
            if self.added and rng.random() < 0.5:
                rid, v, prio = self.added.pop(int(rng.integers(len(self.added))))
                self.log.append({"op": "del", "fid": rid, "side": "src", "addrs": [_ip4(v)], "priority": prio})
                if fast:
                    fast(False, rid, "src", v, prio)
                else:
                    clf.delete_policy_rule_address(rid, "src", [_ip4(v)], prio)
            else:
                r = self.rules[int(rng.integers(len(self.rules)))]
                v = int(rng.integers(0, 1 << 32))
                if fast:
                    fast(True, r["flow_id"], "src", v, r.get("priority"))
                else:
                    clf.add_policy_rule_address(r["flow_id"], "src", [_ip4(v)], r.get("priority"))
                self.added.append((r["flow_id"], v, r.get("priority")))
                self.log.append({"op": "add", "fid": r["flow_id"], "side": "src", "addrs": [_ip4(v)],
                                 "priority": r.get("priority")})
        self.issued += k


VERDICT_NAMES = ("NONE", "NO_MATCH", "ALLOW", "DROP", "REJECT", "ISOLATION_DROP", "BYPASS")


def _verdict_mix(v):
    """Share of each action per stage: v = (n, 2, 8) verdict bytes (byte 4 = action)."""
    import numpy as np
    mix = {}
    for j, stage in enumerate(("egress", "ingress")):
        a, c = np.unique(v[:, j, 4], return_counts=True)
        mix[stage] = {VERDICT_NAMES[int(x)]: round(float(y) / len(v), 4) for x, y in zip(a, c)}
    return mix


def churn_candidates(wl, cols, max_per_packet=1, seed=77):
    """Address adds that change verdicts of the timed batch (C5 "mixed"): for every sampled packet
    (host columns), the rules whose clauses other than the peer clause it matches -- service
    (protocol, destination port in the rule's range) and AppliedTo (ingress: its out_port among the
    rule's ofports; egress: its source among the rule's Pod IPs) -- give (side, flow id, address):
    ingress rules the packet's source as a From peer, egress rules its destination as a To peer.
    Host numpy over the rule set, before the timed region."""
    import numpy as np
    rng = np.random.default_rng(seed)
    m = wl.meta
    n_local = len(wl.local_ips)
    port_ix = {int(p): i for i, p in enumerate(wl.local_ports)}
    ip_ix = {int(a): i for i, a in enumerate(wl.local_ips)}
    nr = len(wl.rules)
    app = np.zeros((nr, n_local), bool)  # AppliedTo of each rule over the local Pods
    for j, r in enumerate(wl.rules):
        if r["direction"] == "In":
            for a in r.get("to") or []:
                if isinstance(a, dict) and "ofport" in a and int(a["ofport"]) in port_ix:
                    app[j, port_ix[int(a["ofport"])]] = True
        else:
            for a in r.get("from") or []:
                if isinstance(a, str) and "/" not in a:
                    v = int.from_bytes(bytes(int(x) for x in a.split(".")), "big")
                    if v in ip_ix:
                        app[j, ip_ix[v]] = True
    d, proto, plo, phi = m["dir"], m["proto"], m["plo"], m["phi"]
    fids = np.array([r["flow_id"] for r in wl.rules])
    out = []
    for i in range(len(cols["src"])):
        p, dp = int(cols["proto"][i]), int(cols["dport"][i])
        svc = (proto == p) & (plo <= dp) & (phi >= dp)
        o = port_ix.get(int(cols["out_port"][i]))
        if o is not None:
            hit = np.nonzero(svc & (d == 0) & app[:, o])[0]
            for j in rng.permutation(hit)[:max_per_packet]:
                out.append(("src", int(fids[j]), int(cols["src"][i])))
        q = ip_ix.get(int(cols["src"][i]))
        if q is not None:
            hit = np.nonzero(svc & (d == 1) & app[:, q])[0]
            for j in rng.permutation(hit)[:max_per_packet]:
                out.append(("dst", int(fids[j]), int(cols["dst"][i])))
    return out


def _ip4(v):
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def _churn_loop(ops, rate, max_batch, stop, rec, interval=0.0):
    """Control-plane thread of C5. Address ops (_ChurnOps) become due at `rate` per second; each
    pass applies every op due so far (at most `max_batch`) and publishes them with one gpc_commit,
    at most one commit per `interval` seconds (the agent's bundle batching: every commit is an
    epoch the data path switches to). Per op, the update latency is the time from the op being due
    to the commit that made it visible returning; rec gets (ops, commit_seconds, [latencies]) per
    commit."""
    import numpy as np
    t0 = time.perf_counter()
    base = ops.issued
    last = t0 - interval
    next_log = t0 + 5.0
    while not stop.is_set():
        now = time.perf_counter()
        if now >= next_log and hasattr(ops.clf, "image_stats"):  # progress (a long C5 run must not look hung)
            next_log = now + 5.0
            st = ops.clf.image_stats()
            _log("C5 %.0f s: %d ops, %d commits (last %.1f ms); journal rules %d, tombstones %d, extended rules %d, "
                 "compactions %d, full builds %d" % (now - t0, ops.issued - base, len(rec), rec[-1][1] * 1e3 if rec else 0,
                                                   st["n_overlay_rules"], st["n_tombstones"], st["n_ext_rules"],
                                                   st["n_background_builds"], st["n_full_builds"]))
        due = int((now - t0) * rate) - (ops.issued - base)
        if due <= 0 or now - last < interval:
            time.sleep(0.0002)
            continue
        last = now
        due = min(due, max_batch)
        first = ops.issued - base
        ops.apply(due)
        tc = time.perf_counter()
        ops.clf.commit()
        done = time.perf_counter()
        due_t = t0 + (first + np.arange(due)) / rate
        rec.append((due, done - tc, done - due_t, now - t0, tc - now))


def _churn_converge(ops, wl, dev, world):
    """After the timed region of C5 at N>1: every rank catches up to the longest op prefix any
    rank applied, commits, and the ranks compare a digest of their realized flows and of their
    device verdicts on one shared packet sample -- the replicated policy is the same everywhere."""
    import hashlib
    import numpy as np
    import torch
    import torch.distributed as dist
    from antrea_amd import workload
    t = torch.tensor([ops.issued], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ops.apply(int(t.item()) - ops.issued)
    ops.clf.commit()
    cols = workload.gen_packets(wl, 1 << 16, seed=4242)
    v = ops.clf.classify_host(cols)
    h = hashlib.sha256("\n".join(ops.clf.dump_flows()).encode())
    h.update(np.ascontiguousarray(v).tobytes())
    mine = torch.tensor(np.frombuffer(h.digest()[:8], np.int64).copy(), device=dev)
    lo, hi = mine.clone(), mine.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return {"ops_applied": int(t.item()), "ranks_identical": bool(lo.item() == hi.item()),
            "digest": h.hexdigest()[:16]}


LAUNCH_KINDS = ("group_tiles", "classify_egress", "classify_ingress", "classify_both", "unpermute", "v6_codes")


def _gather_rank_launch_ms(launches, dev, world):
    """N > 1: every rank's mean HIP-event ms per launch kind of its timed region (gpc_launch_times),
    gathered to every rank in rank order (one all_gather; gloo on CPU in tests)."""
    import torch
    import torch.distributed as dist
    v = torch.tensor([float(launches.get(k, {}).get("mean_ms", -1.0)) for k in LAUNCH_KINDS], dtype=torch.float64,
                     device=dev)
    out = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(out, v)
    return [{k: round(float(x), 3) for k, x in zip(LAUNCH_KINDS, t.cpu().tolist()) if x >= 0} for t in out]


def _pmc_pass(counters, args):
    """One rocprofv3 PMC pass over a short child run of this bench (same workload and packet
    count, counters as configured). Returns {counter: mean value per step} plus the per-kernel
    means ("by_kernel"). Run before this process touches the GPU (the child is a separate
    process, not an exec)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    d = tempfile.mkdtemp(prefix="gpc_pmc_")
    cmd = ["rocprofv3", "--pmc"] + list(counters) + ["--kernel-include-regex", "classify_kernel|group_tiles|unpermute|v6_code_kernel", "-d", d, "-o", "pmc",
                                                       "--output-format", "csv", "--", sys.executable,
                                                       os.path.abspath(__file__), "--steps", "2", "--warmup", "1",
                                                       "--no-cpu-baseline", "--no-traffic", "--no-parity", "--config",
                                                       args.config, "--packets", str(args.packets), "--family",
                                                       str(args.family)]
    if args.no_count:
        cmd.append("--no-count")
    try:
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600, check=True)
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            if args.keep_pmc:  # the raw per-dispatch counter rows behind `roofline` (profiles/)
                os.makedirs(args.keep_pmc, exist_ok=True)
                shutil.copy(f, os.path.join(args.keep_pmc, "pmc_%s_%s.csv" % (args.config, "_".join(counters))))
            with open(f) as fh:
                rows += [r for r in csv.DictReader(fh)
                         if re.search(r"classify_kernel|group_tiles|unpermute|v6_code_kernel", r.get("Kernel_Name", ""))]
        # one step = the grouping launch (if grouped) + two classify launches without Services
        # (egress stage, ingress stage) or one with them (+ the un-permute launch of a grouped batch
        # without Services): steps = dispatches of the first classify stage
        first = [r for r in rows if re.search(r"classify_kernel<\w+, \w+, [01],", r.get("Kernel_Name", ""))]
        steps = len({r.get("Dispatch_Id") for r in first}) or 1
        out, by_kernel = {}, {}
        for c in counters:
            vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == c]
            if vals:
                out[c] = sum(vals) / steps
            for r in rows:
                if r.get("Counter_Name") != c:
                    continue
                k = by_kernel.setdefault(r["Kernel_Name"], {}).setdefault(c, [])
                k.append(float(r["Counter_Value"]))
        out["by_kernel"] = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in by_kernel.items()}
        return out
    except Exception as e:
        print("PMC pass %s failed: %s" % (counters, e), file=sys.stderr)
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _host_sample(cols, idx):
    """Device packet columns -> numpy (unsigned dtypes) at the sample indices."""
    import numpy as np
    import torch
    out = {}
    for k, t in cols.items():
        if t.dtype == getattr(torch, "uint32", None):
            t = t.view(torch.int32)
        a = t[idx].cpu().numpy()
        out[k] = a.view({4: np.uint32, 2: np.uint16, 1: np.uint8}[a.dtype.itemsize])
    return out


def _grouping_label(st, launches, v6):
    """How the timed batches were grouped, from the launches that actually ran (gpc_launch_times)."""
    from antrea_amd import gpc
    if "group_tiles" not in (launches or {}):
        return "off"
    if v6:
        key = "key: top 8 bits of the source address code (IPv6 code columns)"
    elif st["group_key"] == gpc.GROUP_KEY_ADDR:
        sb = int(os.environ.get("GPC_GROUP_SRC_BITS", "8"))
        key = "key: top %d bits of nw_src + %d of nw_dst" % (sb, 8 - sb)
    else:
        key = "key: egress x ingress scan-length bins"
    return key + ", 16384-packet tiles" + (", results un-permuted" if "unpermute" in launches else "")


KIND_STAGE = {"classify_egress": "1", "classify_ingress": "2", "classify_both": "0"}


def _pmc_kernel(by_kernel, kind):
    """PMC means per dispatch of one launch kind (pmc_by_kernel keys are kernel names)."""
    for k, cs in by_kernel.items():
        if kind in ("group_tiles", "unpermute", "v6_codes"):
            if {"v6_codes": "v6_code_kernel"}.get(kind, kind) in k:
                return cs
        else:
            m = re.search(r"classify_kernel<\w+, \w+, (\d)", k)
            if m and m.group(1) == KIND_STAGE.get(kind):
                return cs
    return None


def _traffic(cs):
    """L2 <-> fabric bytes of one launch: FETCH_SIZE x 2 (the gfx950 correction of
    MI355X_MICROARCH.md) + WRITE_SIZE, counters in KB."""
    if not cs or cs.get("FETCH_SIZE") is None or cs.get("WRITE_SIZE") is None:
        return None, None
    return (2.0 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024.0, (cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024.0


def _sq(cs):
    """SQ counters of one launch kind per wave (quad-cycle counters x 4 = cycles)."""
    if not cs or not cs.get("SQ_WAVES"):
        return None
    w = cs["SQ_WAVES"]
    out = {}
    for c, name in (("SQ_INSTS_VMEM_RD", "vmem_rd_per_wave"), ("SQ_INSTS_SALU", "salu_per_wave"),
                    ("SQ_INSTS_VALU", "valu_per_wave")):
        if cs.get(c) is not None:
            out[name] = round(cs[c] / w, 1)
    if cs.get("SQ_WAVE_CYCLES"):
        out["cycles_per_wave"] = round(4.0 * cs["SQ_WAVE_CYCLES"] / w)
        for c, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
            if cs.get(c) is not None:
                out[name] = round(cs[c] / cs["SQ_WAVE_CYCLES"], 3)
    return out


def _roofline(pmc, kern_ms, n, b_in, b_out, lbar, launches):
    """Roofline of the dominant kernel (the launch kind with the largest HIP-event time per step,
    measured on the launch stream inside the timed region: gpc_launch_times), with the whole
    step's figures beside it. Bytes are the measured L2 <-> fabric traffic of the PMC child passes
    (FETCH_SIZE x 2 + WRITE_SIZE per launch; Infinity-Cache hits included, so an upper bound of
    HBM bytes); frac <= 1 is enforced. The x2 FETCH correction is documented for 16-B/lane
    streaming reads; for gathers it is unverified, so the fraction without it is reported too.
    B_alg / L-bar price every image line at HBM cost although most are L2 / MALL
    hits: kept as a diagnostic ("frac_if_uncached" > 1 shows it is not a physical byte count)."""
    by_kernel = {}
    for p in pmc.get("_passes", []):
        for k, cs in (p or {}).get("by_kernel", {}).items():
            short = k.split("(")[0].replace("void gpc::", "")
            by_kernel.setdefault(short, {}).update({c: round(v, 1) for c, v in cs.items()})
    kernels = {}
    for kind, t in (launches or {}).items():
        ms = t["mean_ms"]
        cs = _pmc_kernel(by_kernel, kind)
        tr, tr1 = _traffic(cs)
        d = {"ms": round(ms, 3), "launches_per_step": round(t["per_step"], 2)}
        if tr is not None and ms > 0:
            gbs = tr / (ms / 1e3) / 1e9
            if gbs / HBM_PEAK_GBS > 1.0:
                raise RuntimeError("roofline sanity: %s measured %.0f GB/s exceeds the HBM peak" % (kind, gbs))
            d.update(gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4), bytes_per_packet=round(tr / n, 1),
                     frac_without_fetch_x2=round(tr1 / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4))
        sq = _sq(cs)
        if sq:
            d["sq"] = sq
        kernels[kind] = d
    dom = max(kernels, key=lambda k: kernels[k]["ms"] * kernels[k]["launches_per_step"]) if kernels else None
    rl = {"bound": "hbm", "kernel": dom, "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
          "traffic": None,
          "basis": "dominant kernel: its rocprofv3 FETCH_SIZE*2 + WRITE_SIZE per launch / its mean HIP-event "
                   "duration in the timed region (gpc_launch_times); step: the same over all launches / step time"}
    if dom and "gbs" in kernels[dom]:
        tr, _ = _traffic(_pmc_kernel(by_kernel, dom))
        rl.update(achieved=kernels[dom]["gbs"], frac=kernels[dom]["frac"], traffic=int(tr),
                  kernel_ms=kernels[dom]["ms"], frac_without_fetch_x2=kernels[dom]["frac_without_fetch_x2"])
    if dom and "sq" in kernels[dom]:
        rl["sq"] = kernels[dom]["sq"]
    rl["kernels"] = kernels
    step = {"ms": round(kern_ms, 3)}
    f, w = pmc.get("FETCH_SIZE"), pmc.get("WRITE_SIZE")
    if f is not None and w is not None:
        traffic = (2.0 * f + w) * 1024.0
        gbs = traffic / (kern_ms / 1e3) / 1e9
        if gbs / HBM_PEAK_GBS > 1.0:
            raise RuntimeError("roofline sanity: measured %.0f GB/s exceeds the HBM peak" % gbs)
        step.update(achieved=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4), traffic=int(traffic),
                    traffic_per_packet=round(traffic / n, 1))
    hit, miss = pmc.get("TCC_HIT_sum"), pmc.get("TCC_MISS_sum")
    if hit is not None and miss is not None and hit + miss > 0:
        step["l2_hit_rate"] = round(hit / (hit + miss), 4)
        step["l2_miss_bytes_per_packet"] = round(miss * 128.0 / n, 1)  # 128-B L2 lines
    rl["step"] = step
    pps_kernel = n / (kern_ms / 1e3)
    b_alg = b_in + b_out + (64.0 * lbar if lbar is not None else 0.0)
    rl["algorithmic"] = {"bytes_per_packet": round(b_alg, 1), "lines_per_packet": round(lbar, 2) if lbar else None,
                         "gbs_if_uncached": round(pps_kernel * b_alg / 1e9, 1),
                         "frac_if_uncached": round(pps_kernel * b_alg / 1e9 / HBM_PEAK_GBS, 4),
                         "compulsory_bytes_per_packet": b_in + b_out,
                         "compulsory_frac": round(pps_kernel * (b_in + b_out) / 1e9 / HBM_PEAK_GBS, 4)}
    rl["pmc_by_kernel"] = by_kernel or None
    return rl


class _HipPath:
    """The product data path of one rank: gpc_classify* on this rank's GPU (the HIP kernels of
    libgpc.so), timed with HIP events on the launch stream, counters all-reduced over RCCL."""
    label = None

    def __init__(self, local):
        import torch
        self.torch = torch
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)

    def init_dist(self):
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=self.dev)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def stream(self, own):
        return self.torch.cuda.Stream(self.dev) if own else self.torch.cuda.current_stream(self.dev)

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)

    def bind(self, clf, v6):
        self.clf = clf
        self.fn = clf.classify6_device if v6 else clf.classify_device

    def commit(self):
        self.clf.commit()

    def classify(self, soa, n, out, count, stream):
        self.fn(soa, n, out.data_ptr(), count=count, stream=stream.cuda_stream)

    def reset_counters(self):
        self.clf.reset_counters()

    def set_launch_timing(self, k):
        self.clf.set_launch_timing(k)

    def launch_times(self):
        return self.clf.launch_times()

    def counters(self):
        """The library's device counters, wrapped zero-copy (None when counting is off)."""
        from antrea_amd import dist as gdist
        ptr, slots = self.clf.counters()
        return gdist.device_counters(ptr, len(slots), self.dev) if ptr and slots else None


class _HostEmuPath(_HipPath):
    """TEST-ONLY stand-in for _HipPath (GPC_BENCH_HOST_EMU=1; tests/test_bench_host.py): runs
    bench's multi-rank plumbing -- rank launch, gloo rendezvous, per-rank launch times, counter
    all-reduce, rank-0 parity stamp -- on a host without a GPU. The classify call is the host
    emulation of the same committed image (tests/emu: core.hpp compiled with g++), so the parity
    stamp is still a real comparison. Refuses to run where a GPU is visible, and the line says
    data: "host-emulation test stub": it is never a measurement."""
    label = "host-emulation test stub (not a measurement)"

    def __init__(self, local):
        import torch
        if torch.cuda.is_available():
            raise SystemExit("GPC_BENCH_HOST_EMU is a CPU test hook; unset it on a GPU host")
        from tests import emu
        self.torch, self.emu = torch, emu
        self.dev = torch.device("cpu")
        self.times = []
        self.timing = 0
        self.cnt = None

    def init_dist(self):
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def sync(self):
        pass

    def stream(self, own):
        return None

    def event(self):
        class Ev:
            def record(self, stream=None):
                self.t = time.perf_counter()

            def elapsed_time(self, other):
                return (other.t - self.t) * 1e3
        return Ev()

    def bind(self, clf, v6):
        if v6:
            raise SystemExit("GPC_BENCH_HOST_EMU: IPv4 only")
        self.clf = clf

    def commit(self):
        self.emu.commit_host(self.clf)
        n = self.clf.image_stats()["n_counter_slots"]
        if self.cnt is None or len(self.cnt) < 3 * n:
            self.cnt = self.torch.zeros(3 * max(1, n), dtype=self.torch.int64)

    def classify(self, soa, n, out, count, stream):
        import numpy as np
        from antrea_amd import gpc
        t0 = time.perf_counter()
        cols = {}
        for name, dt in gpc.PKT_COLUMNS.items():
            p = getattr(soa, name)
            if p:
                cols[name] = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                                   shape=(n,))
        c = self.cnt.numpy().view(np.uint64) if count else None
        v = self.emu.classify(self.clf, cols, counters=c)
        out.numpy()[:] = np.ascontiguousarray(v).view(np.uint8).reshape(-1)
        if self.timing and len(self.times) < self.timing:
            self.times.append((time.perf_counter() - t0) * 1e3)

    def reset_counters(self):
        self.cnt.zero_()

    def set_launch_timing(self, k):
        self.timing, self.times = k, []

    def launch_times(self):
        if not self.times:
            return {}
        return {"classify_both": {"launches": len(self.times), "total_ms": sum(self.times),
                                  "mean_ms": sum(self.times) / len(self.times), "dropped": 0}}

    def counters(self):
        return self.cnt


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK,
    LOCAL_RANK = GPU ordinal, WORLD_SIZE, MASTER_ADDR / a free MASTER_PORT), as
    torch.distributed.run would. This process never imports torch nor touches a GPU (no exec:
    the ranks are children). Rank 0's JSON line is printed; the first rank to fail stops the
    others and its exit code is returned."""
    import subprocess
    import tempfile
    port = _free_port()
    procs = []
    out0 = tempfile.TemporaryFile(mode="w+")
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out0 if r == 0 else sys.stderr.fileno()))
    _log("launched %d ranks (pids %s, port %d)" % (n, [p.pid for p in procs], port))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                _log("rank %d exited with %d: stopping the others" % (procs.index(p), code))
                for q in live:
                    q.kill()
    out0.seek(0)
    for line in out0.read().splitlines():  # the JSON line to stdout, anything a library printed to stderr
        if rc == 0 and line.startswith("{"):
            print(line, flush=True)
        else:
            print(line, file=sys.stderr)
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="N GPUs of this node, one rank per GPU (default: WORLD_SIZE, else 1); without a "
                         "launcher bench.py starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--no-count", action="store_true", help="disable per-rule counters")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the timed batch")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC child passes")
    ap.add_argument("--keep-pmc", default="", help="directory that keeps the PMC passes' counter CSVs")
    ap.add_argument("--churn-rate", type=float, default=10000.0, help="C5: address ops per second")
    ap.add_argument("--max-batch", type=int, default=2000, help="C5: most address ops per gpc_commit")
    ap.add_argument("--churn-mix", default="mixed", choices=("mixed", "uniform"),
                    help="C5 op stream: mixed = adds of peers the batch sends + base-peer deletes / re-adds + "
                         "uninstall / reinstall + priority reassignment (_ChurnOps.MIX); uniform = round 5's "
                         "random /32 source adds / deletes")
    ap.add_argument("--churn-base-frac", type=float, default=0.005,
                    help="C5 mixed: share of ops that delete / re-add a rule's own ipBlock peers (policy edits: "
                         "journaled; 0.005 = 50 / s at 10 000 ops / s)")
    ap.add_argument("--commit-interval-ms", type=float, default=10.0,
                    help="C5: at most one gpc_commit per this many ms (ops due meanwhile share it)")
    ap.add_argument("--compact-after", type=int, default=0,
                    help="gpc_config.compact_after: live journal rules that start a background compaction "
                         "(0 = the library default, max(512, base rules / 128))")
    ap.add_argument("--group", type=int, default=0,
                    help="gpc_config.group_packets: 0 = auto (batches >= 2^18 against images >= 4 MB), 1 = on, -1 = off")
    ap.add_argument("--family", type=int, default=4, choices=(4, 6),
                    help="6: the workload's addresses embedded in fd00:10::/96, IPv6 packets (gpc_classify6)")
    ap.add_argument("--v6-embed", default="96", choices=("96", "multi48"),
                    help="--family 6: fd00:10::/96, or four /48s chosen by the top 2 IPv4 bits (workload.v6_embed)")
    ap.add_argument("--multidev", type=int, default=0,
                    help="one process over N devices (gpc_create_multi: the agent's shape, one control plane per "
                         "node) instead of one process per GPU; N slots, one stream and host thread per slot")
    ap.add_argument("--multidev-devices", default="",
                    help="HIP ordinals of the --multidev slots (default 0..N-1; e.g. 0,0 = two slots on one GPU)")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)
    if args.multidev:
        return main_multidev(args)
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is not None and args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%s (one rank per GPU)" % (args.gpus, env_world), file=sys.stderr)
        return 2
    if env_world is None and (args.gpus or 1) > 1:
        return launch_ranks(args.gpus, argv)
    if args.family == 6 and args.config in ("C4", "C5"):
        ap.error("--family 6: C1-C3 only (no IPv6 AntreaProxy stage / delta epochs)")
    churn = args.config == "C5"
    if churn:  # the timed batch sees many epochs: parity is checked on the final epoch (below)
        args.no_traffic = True
        args.no_cpu_baseline = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host_emu = os.environ.get("GPC_BENCH_HOST_EMU") == "1"
    if world > 1 or host_emu:  # the CPU baseline is an N=1 figure; every N still gets rank 0's parity stamp
        args.no_cpu_baseline = True
    if host_emu:
        args.no_traffic = True
    worker = None
    if rank == 0 and not (args.no_parity and args.no_cpu_baseline):
        # the CPU oracle (oracle compiler + C classifier) is prepared in a spawned process while
        # this one profiles and times the GPU; it never touches the GPU. C5: it keeps the oracle
        # compiler and later replays the op log the run applied.
        from oracle.parity import OracleWorker
        worker = OracleWorker("C3" if churn else args.config, churn=churn)

    import torch
    import torch.distributed as dist

    pmc = {}
    if world == 1 and not args.no_traffic:
        passes = []
        for c in PMC_PASSES:
            _log("rocprofv3 PMC pass %s" % " ".join(c))
            passes.append(_pmc_pass(c, args))
        for p in passes:
            pmc.update({k: v for k, v in (p or {}).items() if k != "by_kernel"})
        pmc["_passes"] = passes
    dp = (_HostEmuPath if host_emu else _HipPath)(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dp.init_dist()
    dev = dp.dev

    from antrea_amd import gpc, workload
    from antrea_amd.build import build
    if rank == 0 or world == 1:
        build()
    if world > 1:
        dist.barrier()

    _log("building the %s rule set" % args.config)
    t0 = time.time()
    wl = workload.CONFIGS["C3" if churn else args.config]()
    v6 = args.family == 6
    clf = gpc.Classifier(device=local, ipv4=not v6, ipv6=v6, group_packets=args.group, compact_after=args.compact_after)
    dp.bind(clf, v6)
    clf.initialize()
    clf.batch_install_policy_rule_flows(workload.to_ipv6(wl, embed=args.v6_embed).rules if v6 else wl.rules)
    if getattr(wl, "services", None):
        workload.install_services(clf, wl)
    dp.commit()
    t_build = time.time() - t0

    n = args.packets
    cols4 = workload.gen_packets_torch(wl, n, seed=workload.PKT_SEED + rank, device=dev)
    cols = workload.packets_to_v6_torch(cols4, embed=args.v6_embed) if v6 else cols4
    out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
    soa = gpc.pkt_soa_device(cols)
    count = not args.no_count
    stream = dp.stream(own=churn)
    for _ in range(args.warmup):
        dp.classify(soa, n, out, count, stream)
    dp.reset_counters()
    dp.sync()
    if world > 1:
        dist.barrier()
    dp.sync()
    starts = [dp.event() for _ in range(args.steps)]
    ends = [dp.event() for _ in range(args.steps)]
    lat, th = [], None
    # The harness's own heap (the workload's 100 k rule dicts, C5's op log growing by 10 k dicts a
    # second) makes CPython's cyclic collector pause every thread for up to ~0.6 s while it holds
    # the GIL: the launch loop stalled (C5 step max 564 ms, op p99 680 ms). Nothing of the library
    # is collected; the harness freezes its heap (before the control thread starts: the collection itself
    # holds the GIL for ~0.3 s) and collects again after the timed region.
    import gc
    gc.collect()
    gc.freeze()
    gc.disable()
    if churn:
        import threading
        import numpy as np
        # the C3 verdicts of the batch prefix (warmup ran on the base epoch): the mix shift baseline
        n_pre = min(n, 1 << 20)
        v_before = out.view(torch.uint8).reshape(n, 2, 8)[:n_pre].cpu().numpy().copy()
        cands = None
        if args.churn_mix == "mixed":
            # adds that hit the timed batch: candidates from rank 0's batch prefix (every rank derives
            # the same list, so every rank applies the same op stream)
            k_c = min(n_pre, 8192)
            idx_c = (torch.arange(k_c, dtype=torch.int64) * n_pre) // k_c
            c0 = cols4 if rank == 0 else workload.gen_packets_torch(wl, n, seed=workload.PKT_SEED, device=dev)
            cands = churn_candidates(wl, _host_sample(c0, idx_c.to(dev)))
            del c0
            _log("C5 mixed: %d candidate adds from %d sampled packets" % (len(cands), k_c))
        st0 = clf.image_stats()
        sys.setswitchinterval(2e-4)  # the control thread must not wait 5 ms for the GIL behind launches
        stop = threading.Event()
        churn_ops = _ChurnOps(clf, wl, seed=1234, mix=args.churn_mix, cands=cands,
                              base_frac=args.churn_base_frac)  # the same op stream on every rank
        th = threading.Thread(target=_churn_loop, args=(churn_ops, args.churn_rate, args.max_batch, stop, lat,
                                                        args.commit_interval_ms / 1e3), daemon=True)
        th.start()
        while len(lat) < 5:  # control loop running before the timed region
            time.sleep(0.01)
        lat.clear()
    _log("timed region: %d steps of %d packets" % (args.steps, n))
    # HIP events around each kernel of the timed calls (gpc_launch_times; the library keeps at most
    # 4096 calls: a longer run, e.g. C5 over 30 s, is timed per kernel over its first 4096 steps)
    dp.set_launch_timing(min(args.steps, 4096))
    dp.sync()
    t_start = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        dp.classify(soa, n, out, count, stream)
        ends[i].record(stream)
        if churn and i % 1000 == 999:  # progress of a long C5 run (launches are paced: ~the device's rate)
            _log("C5: %d steps launched" % (i + 1))
    dp.sync()
    if world > 1:
        dist.barrier()
    dp.sync()
    elapsed = time.perf_counter() - t_start
    update = None
    if churn:
        stop.set()
        th.join()
        import numpy as np
        rec = lat[:]
        ops = sum(r[0] for r in rec)
        op_ms = np.concatenate([r[2] for r in rec]) * 1e3 if rec else np.zeros(0)
        commit_ms = np.array([r[1] for r in rec]) * 1e3
        st = clf.image_stats()
        pct = lambda a, q: round(float(np.percentile(a, q)), 3) if len(a) else None
        update = {"ops": int(ops), "commits": len(rec), "ops_per_s": round(ops / elapsed, 1),
                  "target_ops_per_s": args.churn_rate, "ops_per_commit_mean": round(ops / max(1, len(rec)), 1),
                  "commit_interval_ms": args.commit_interval_ms, "timed_s": round(elapsed, 2),
                  "op_latency_ms": {"p50": pct(op_ms, 50), "p99": pct(op_ms, 99),
                                    "max": round(float(op_ms.max()), 3) if len(op_ms) else None},
                  "commit_ms": {"p50": pct(commit_ms, 50), "p99": pct(commit_ms, 99)},
                  # the commit whose ops waited longest: when it ran (seconds into the control loop),
                  # how long applying its ops and the commit took
                  "worst_commit": (lambda r: {"at_s": round(r[3], 3), "ops": int(r[0]), "apply_ms": round(r[4] * 1e3, 2),
                                              "commit_ms": round(r[1] * 1e3, 2),
                                              "op_latency_ms": round(float(r[2].max()) * 1e3, 2)})(
                      max(rec, key=lambda r: float(r[2].max()))) if rec else None,
                  "overlay_rules_end": st["n_overlay_rules"], "tombstones_end": st["n_tombstones"],
                  "ext_rules_end": st["n_ext_rules"], "ext_values_end": st["n_ext_values"],
                  "full_builds": st["n_full_builds"] - st0["n_full_builds"],
                  "delta_builds": st["n_delta_builds"] - st0["n_delta_builds"],
                  "background_builds": st["n_background_builds"] - st0["n_background_builds"],
                  "mix": args.churn_mix}
        if args.churn_mix == "mixed":
            update["op_counts"] = dict(churn_ops.counts)
            update["candidate_adds"] = len(cands)
        if world > 1:
            update["ranks"] = _churn_converge(churn_ops, wl, dev, world)
    gc.enable()  # (after the control thread stopped: the op log's first collection is long)
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps
    launches = dp.launch_times()
    dp.set_launch_timing(0)
    for t in launches.values():
        t["per_step"] = t["launches"] / args.steps
    rank_launches = _gather_rank_launch_ms(launches, dev, world) if world > 1 else None
    if churn and worker is not None and not args.no_parity:
        # parity of C5: the oracle replays the op prefix this rank applied (every op was committed
        # before the control thread stopped), and the final epoch classifies the batch once more
        _log("oracle replay of %d ops" % len(churn_ops.log))
        update["oracle_replay"] = worker.churn(churn_ops.log)
    if churn:
        # step times over the timed region (is the cost steady or in bursts?) and the final epoch
        # timed alone, with the control thread stopped (epoch state vs concurrent commits)
        import numpy as np
        step_ms = np.array([s_.elapsed_time(e_) for s_, e_ in zip(starts, ends)])
        w = max(1, len(step_ms) // 16)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(10):
            dp.classify(soa, n, out, count, stream)
        ev[1].record(stream)
        dp.sync()
        st_end = clf.image_stats()
        update["step_ms"] = {"p50": round(float(np.percentile(step_ms, 50)), 3),
                             "p90": round(float(np.percentile(step_ms, 90)), 3),
                             "max": round(float(step_ms.max()), 3),
                             "windows": [round(float(step_ms[i:i + w].mean()), 2) for i in range(0, len(step_ms), w)],
                             "final_epoch_alone": round(ev[0].elapsed_time(ev[1]) / 10, 3),
                             "final_epoch_mode": {"journal_rules": st_end["n_overlay_rules"],
                                                  "ext_rules": st_end["n_ext_rules"]}}
    if churn:  # the final epoch classifies the batch once more (parity sample, verdict shift)
        dp.classify(soa, n, out, False, stream)
        dp.sync()
        v_after = out.view(torch.uint8).reshape(n, 2, 8)[:n_pre].cpu().numpy()
        changed = (v_before.reshape(n_pre, 16) != v_after.reshape(n_pre, 16)).any(axis=1)
        update["verdict_shift"] = {
            "packets": n_pre, "changed_frac": round(float(changed.mean()), 6),
            "mix_before": _verdict_mix(v_before), "mix_after": _verdict_mix(v_after),
            "basis": "verdicts of the first %d packets on the base (C3) epoch, before the churn, vs on the final "
                     "epoch" % n_pre}
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    counters_reduced = None
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # per-rule counters: the path's only collective (RCCL all-reduce). The
        # library's device counters are wrapped zero-copy and reduced in place.
        cnt = dp.counters() if count else None
        if cnt is not None:
            from antrea_amd import dist as gdist
            dp.sync()
            gdist.allreduce_counters(cnt)
            dp.sync()
            counters_reduced = {"slots": len(cnt) // 3, "packets": int(cnt.view(-1, 3)[:, 0].sum().item())}
    elapsed = float(t.item())

    total = n * args.steps * world
    mpps = total / elapsed / 1e6
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return 0

    import numpy as np
    from antrea_amd.gpc import VERDICT_DTYPE
    v8 = out.view(torch.uint8).reshape(n, 2, 8)
    mix = _verdict_mix(v8[: min(n, 1 << 20)].cpu().numpy())

    parity = None
    if worker is not None and not args.no_parity:  # rank 0 (its own shard at N > 1)
        k = min(n, PARITY_SAMPLE)
        idx_h = (torch.arange(k, dtype=torch.int64) * n) // k  # integer stride: every index < n
        assert int(idx_h.max()) < n and int(idx_h.min()) >= 0
        idx = idx_h.to(dev)
        sample = _host_sample(cols4, idx)
        got = np.ascontiguousarray(v8[idx].cpu().numpy()).view(VERDICT_DTYPE).reshape(-1, 2)
        _log("parity check of %d sampled packets (waiting for the oracle process)" % len(idx))
        parity = worker.check(sample, got)
        parity["sample"] = "%d packets, stride %.0f over the timed batch (%s)%s%s" % (
            len(idx), n / len(idx),
            "classified again on the final epoch, vs the oracle after replaying the %d applied ops" % len(churn_ops.log)
            if churn else "last step's verdicts",
            "; IPv6 packets vs the IPv4 oracle (%s embedding)" % ("fd00:10::/96" if args.v6_embed == "96" else
                                                                 "four /48s") if v6 else "",
            "; rank 0's shard of %d" % world if world > 1 else "")
        if parity.get("mismatches"):
            print("PARITY FAILURE: %s" % json.dumps(parity), file=sys.stderr)

    lbar = _lbar(wl, clf, family=args.family)
    b_in, b_out = (19 if getattr(wl, "services", None) else 17), 16  # +2 B len for C4
    if v6:
        b_in += 24  # 16-B instead of 4-B src / dst
    roofline = _roofline(pmc, kern_ms, n, b_in, b_out, lbar, launches)
    cpu = None
    if worker is not None and not args.no_cpu_baseline:  # rank 0, N=1 only
        _log("CPU baseline (%.0f s)" % args.cpu_seconds)
        cpu = worker.baseline(args.cpu_seconds)
    if worker is not None:
        worker.close()
    st = clf.image_stats()
    res = {
        "metric": "Mpps classified (5-tuple->rule verdict) @100k rules, 1-8 MI355X; % HBM BW",
        "value": round(mpps, 2), "unit": "Mpps", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": dp.label or "synthetic",
        "config": {"workload": args.config, "rules": len(wl.rules), "packets_per_gpu": n,
                   "flows": st["n_flows"],
                   "image_mb": round((clf.debug_image6()[1] * 4 if v6 else st["device_bytes"]) / 1e6, 1),
                   "counters": count, "parallelism": "packet-shard x%d, rules replicated" % world,
                   "verdict_mix": mix, "build_s": round(t_build, 1),
                   "packet_grouping": _grouping_label(st, launches, v6)},
        "kernel_ms": round(kern_ms, 3),  # all launches of a step (HIP events on the launch stream)
        "launches_per_step": round(sum(t["per_step"] for t in launches.values()), 2),
        "kernel_ms_by_launch": {k: round(t["mean_ms"], 3) for k, t in launches.items()},
        "kernel_ms_by_launch_per_rank": rank_launches,
        "counters_allreduced": counters_reduced,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if getattr(wl, "services", None):
        res["metric"] = "Mpps classified (AntreaProxy ServiceLB/EndpointDNAT + policy) @100k rules, 10k Services"
        res["config"]["services"] = len(wl.services)
        res["config"]["endpoints"] = sum(len(e) for e in wl.groups.values())
        res["config"]["to_service_frac"] = wl.svc_frac
    if v6:
        res["metric"] = "Mpps classified (IPv6 5-tuple->rule verdict) @100k rules, 1-8 MI355X; % HBM BW"
        res["config"]["family"] = 6
        res["config"]["v6_embedding"] = "fd00:10::/96" if args.v6_embed == "96" else "fd00:0:k::/48, k = top 2 bits"
    if update is not None:
        res["update"] = update
        res["metric"] = "Mpps classified under AddPolicyRuleAddress/DeletePolicyRuleAddress churn @100k rules"
    print(json.dumps(res))
    sys.stdout.flush()
    if world > 1:
        dist.destroy_process_group()
    return 0


def main_multidev(args):
    """bench.py --multidev N: one process, one gpc context over N device slots (gpc_create_multi),
    as the agent runs it (one control plane per node, cmd/antrea-agent/agent.go:177). Every slot
    holds the same epoch; each classifies its own packet shard (weak scaling: --packets per slot)
    on its own stream, driven by its own host thread; the per-rule counters of all slots are summed
    in-process by gpc_metrics (the in-process counterpart of the RCCL all-reduce). Same JSON line
    schema; value = packets of all slots / the wall time of the timed region."""
    import threading
    import numpy as np
    import torch
    from antrea_amd import gpc, workload
    from antrea_amd.build import build
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--multidev runs as one process (not under torchrun)")
    if args.config in ("C5",) or args.family != 4:
        raise SystemExit("--multidev: C1-C4, IPv4")
    n_slots = args.multidev
    devs = [int(x) for x in args.multidev_devices.split(",")] if args.multidev_devices else list(range(n_slots))
    if len(devs) != n_slots:
        raise SystemExit("--multidev-devices lists %d ordinals for %d slots" % (len(devs), n_slots))
    worker = None
    if not (args.no_parity and args.no_cpu_baseline):
        from oracle.parity import OracleWorker
        worker = OracleWorker(args.config)
    build()
    _log("building the %s rule set (one context, %d slots on devices %s)" % (args.config, n_slots, devs))
    t0 = time.time()
    wl = workload.CONFIGS[args.config]()
    clf = gpc.Classifier(devices=devs, group_packets=args.group)
    clf.initialize()
    clf.batch_install_policy_rule_flows(wl.rules)
    if getattr(wl, "services", None):
        workload.install_services(clf, wl)
    clf.commit()  # published on every slot
    t_build = time.time() - t0
    n = args.packets
    count = not args.no_count
    slots = []
    for k, d in enumerate(devs):
        dev = torch.device("cuda", d)
        with torch.cuda.device(dev):
            cols = workload.gen_packets_torch(wl, n, seed=workload.PKT_SEED + k, device=dev)
            slots.append({"dev": dev, "cols": cols, "soa": gpc.pkt_soa_device(cols),
                          "out": torch.empty(2 * n * 8, dtype=torch.uint8, device=dev),
                          "stream": torch.cuda.Stream(dev)})

    def run(k, steps, evs=None):
        sl = slots[k]
        with torch.cuda.device(sl["dev"]):
            for i in range(steps):
                if evs is not None:
                    evs[k][0][i].record(sl["stream"])
                clf.classify_device(sl["soa"], n, sl["out"].data_ptr(), count=count, stream=sl["stream"].cuda_stream,
                                    slot=k)
                if evs is not None:
                    evs[k][1][i].record(sl["stream"])

    def all_slots(steps, evs=None):
        th = [threading.Thread(target=run, args=(k, steps, evs)) for k in range(n_slots)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    def sync():
        for sl in slots:
            torch.cuda.synchronize(sl["dev"])

    all_slots(args.warmup)
    sync()
    clf.reset_counters()
    sync()
    evs = [([torch.cuda.Event(enable_timing=True) for _ in range(args.steps)],
            [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]) for sl in slots]
    _log("timed region: %d steps x %d slots of %d packets" % (args.steps, n_slots, n))
    t_start = time.perf_counter()
    all_slots(args.steps, evs)
    sync()
    elapsed = time.perf_counter() - t_start
    slot_ms = [sum(a.elapsed_time(b) for a, b in zip(*evs[k])) / args.steps for k in range(n_slots)]
    total = n * args.steps * n_slots
    metrics = clf.network_policy_metrics() if count else {}
    parity = None
    if worker is not None and not args.no_parity:
        from antrea_amd.gpc import VERDICT_DTYPE
        k_s = min(n, PARITY_SAMPLE // n_slots or 1)
        res = []
        for k, sl in enumerate(slots):
            idx_h = (torch.arange(k_s, dtype=torch.int64) * n) // k_s
            idx = idx_h.to(sl["dev"])
            sample = _host_sample(sl["cols"], idx)
            v8 = sl["out"].view(torch.uint8).reshape(n, 2, 8)
            got = np.ascontiguousarray(v8[idx].cpu().numpy()).view(VERDICT_DTYPE).reshape(-1, 2)
            res.append(worker.check(sample, got))
        parity = {"checked": sum(r["checked"] for r in res), "mismatches": sum(r["mismatches"] for r in res),
                  "sample": "%d packets per slot, stride %.0f over each slot's timed batch" % (k_s, n / k_s)}
        if parity["mismatches"]:
            print("PARITY FAILURE: %s" % json.dumps(res), file=sys.stderr)
    cpu = None
    if worker is not None and not args.no_cpu_baseline:
        cpu = worker.baseline(args.cpu_seconds)
    if worker is not None:
        worker.close()
    st = clf.image_stats()
    res = {
        "metric": "Mpps classified (5-tuple->rule verdict) @100k rules, 1-8 MI355X; % HBM BW",
        "value": round(total / elapsed / 1e6, 2), "unit": "Mpps", "n_gpus": len(set(devs)), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": args.config, "rules": len(wl.rules), "packets_per_slot": n, "slots": n_slots,
                   "devices": devs, "flows": st["n_flows"], "counters": count, "build_s": round(t_build, 1),
                   "parallelism": "one process, gpc_create_multi over %d device slots (packet shards, one epoch "
                                  "published on every slot)" % n_slots},
        "slot_kernel_ms": [round(x, 3) for x in slot_ms],
        "metrics_rules_nonzero": sum(1 for v in metrics.values() if any(v)),
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if getattr(wl, "services", None):
        res["metric"] = "Mpps classified (AntreaProxy ServiceLB/EndpointDNAT + policy) @100k rules, 10k Services"
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
