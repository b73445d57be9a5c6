"""Oracle verdicts for whole workloads (TEST / MEASUREMENT INFRASTRUCTURE ONLY).

* `oracle_pipeline(wl)`   -- the C restatement of the OVS classifier (ovs_cls.c) loaded with the
                             flows the ORACLE compiler (oracle/compiler.py) emits for `wl.rules`;
                             never the product compiler's dump, so a product compiler bug cannot
                             hide on both sides of a comparison.
* `oracle_metrics(pipe)`  -- NetworkPolicyMetrics of the counters the C oracle accumulated
                             (parsed exactly as network_policy.go:1917-1980, 2034 parse the dump).
* `service_flows(wl)`     -- for a workload with Services (C4): the ServiceLB / EndpointDNAT flow
                             text, the select groups and the Pod map the C oracle's AntreaProxy stage
                             runs on, from the oracle's own restatement of the Service flows
                             (oracle/service.py, pinned by the reference's client_test.go goldens;
                             equal to the product's dumps, tests/test_service.py).
Nothing here loads the product library or its compiler; `antrea_amd.workload` (the synthetic
input generator shared with bench.py) is the only import from the product package.
* `non_service_mask`      -- packets of a workload with Services that do not hit a ServiceLB flow.
* `OracleWorker`          -- the same in a separate CPU process (spawned, never touches a GPU):
                             bench.py starts it before its GPU work, then asks it to check a sample
                             of the timed batch (parity stamp) and to time the CPU baseline.
"""
from __future__ import annotations

import copy
import os
import platform
import time
from typing import Dict, Optional

import numpy as np

VERDICT_NP = np.dtype([("conj_id", "<u4"), ("action", "u1"), ("table", "u1"), ("tier", "u1"), ("flags", "u1")])


def cpu_threads() -> int:
    """Threads of the CPU legs: the process's CPU share (OMP_NUM_THREADS when the box sets it,
    else the CPUs this process may run on)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def host_info() -> dict:
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model}


def tiers_of(wl) -> Dict[int, int]:
    return {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}


def oracle_flows(wl):
    from . import compiler as oc
    fnp = oc.FeatureNetworkPolicy()
    fnp.initialize()
    fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    return fnp.dump_flows()


def service_flows(wl):
    """(ServiceLB / EndpointDNAT flow lines, group lines, Pod map) of wl's Services, or None: the
    oracle's own restatement of the AntreaProxy flows (oracle/service.py, pinned by the
    client_test.go goldens), not the product's compiler."""
    if getattr(wl, "services", None) is None:
        return None
    from . import service as osvc
    s = osvc.FeatureService()
    osvc.install_services(s, wl)
    lines = [f for f in s.dump_flows() if "table=ServiceLB" in f or "table=EndpointDNAT" in f]
    return lines, s.dump_groups(), dict(wl.pods)


def oracle_pipeline(wl, procs: Optional[int] = None, flows=None):
    from .cls_c import CPipeline
    svc = service_flows(wl)
    pipe = CPipeline((oracle_flows(wl) if flows is None else flows) + (svc[0] if svc else []), tiers_of(wl), procs=procs)
    if svc:
        pipe.set_services(svc[1], svc[2])
    return pipe


def _ip4(v: int) -> str:
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def replay_churn(fnp, ops) -> int:
    """Apply bench.py's C5 op log to the oracle compiler, in the order the product applied it. Ops
    are dicts (bench._ChurnOps): {"op": "add" | "del", "fid", "side", "addrs", "priority"}
    (AddPolicyRuleAddress / DeletePolicyRuleAddress, network_policy.go:1661-1710), {"op":
    "uninstall", "fid"} (UninstallPolicyRuleFlows :1570), {"op": "install", "rule"}
    (InstallPolicyRuleFlows :1160), {"op": "reassign", "table", "from", "to"}
    (ReassignFlowPriorities :1873). Round 5's tuples (kind 1 = add / 0 = delete, rule id, IPv4
    value, priority or -1) of one /32 source peer are still accepted."""
    for o in ops:
        if not isinstance(o, dict):
            kind, rid, v, prio = o
            prio = None if prio is None or prio < 0 else int(prio)
            o = {"op": "add" if kind else "del", "fid": int(rid), "side": "src", "addrs": [_ip4(int(v))],
                 "priority": prio}
        k = o["op"]
        if k == "add":
            fnp.add_policy_rule_address(o["fid"], o["side"], copy.deepcopy(o["addrs"]), o["priority"])
        elif k == "del":
            fnp.delete_policy_rule_address(o["fid"], o["side"], copy.deepcopy(o["addrs"]), o["priority"])
        elif k == "uninstall":
            fnp.uninstall_policy_rule_flows(o["fid"])
        elif k == "install":
            fnp.install_policy_rule_flows(copy.deepcopy(o["rule"]))
        elif k == "reassign":
            fnp.reassign_flow_priorities({o["from"]: o["to"]}, o["table"])
        else:
            raise ValueError("unknown churn op %r" % (k,))
    return len(ops)


def oracle_metrics(pipe) -> Dict[int, tuple]:
    from . import compiler as oc
    d = pipe.metric_dumps()
    return oc.network_policy_metrics(d["EgressMetric"], d["IngressMetric"])


def non_service_mask(wl, cols) -> np.ndarray:
    """True for packets that match no ServiceLB flow of wl (proto, Service IP, port)."""
    sm = getattr(wl, "svc_meta", None)
    n = len(cols["src"])
    if sm is None:
        return np.ones(n, bool)
    keys = set(zip(sm["proto"].astype(np.int64).tolist(), sm["ip"].astype(np.int64).tolist(),
                   sm["port"].astype(np.int64).tolist()))
    p, d, dp = (cols[k].astype(np.int64).tolist() for k in ("proto", "dst", "dport"))
    return np.array([(a, b, c) not in keys for a, b, c in zip(p, d, dp)], bool)


def compare(got: np.ndarray, want: np.ndarray, mask: Optional[np.ndarray] = None) -> dict:
    """Packet-for-packet verdict comparison: (n, 2) verdict records (8 B each)."""
    g = np.ascontiguousarray(got).view(np.uint64).reshape(-1, 2)
    w = np.ascontiguousarray(want).view(np.uint64).reshape(-1, 2)
    idx = np.arange(len(g)) if mask is None else np.nonzero(mask)[0]
    bad = idx[(g[idx] != w[idx]).any(axis=1)]
    res = {"checked": int(len(idx)), "mismatches": int(len(bad))}
    if len(bad):
        i = int(bad[0])
        res["first"] = {"index": i, "device": [int(x) for x in g[i]], "oracle": [int(x) for x in w[i]]}
    return res


# ------------------------------------------------------------------------------ worker process
def _serve(conn, config: str, procs: int, churn: bool = False):
    from antrea_amd import workload
    from . import compiler as oc
    t0 = time.time()
    wl = workload.CONFIGS[config]()
    fnp = None
    if churn:  # keep the oracle compiler: the op log of the run is replayed on it afterwards
        fnp = oc.FeatureNetworkPolicy()
        fnp.initialize()
        fnp.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
        pipe = oracle_pipeline(wl, procs=procs, flows=fnp.dump_flows())
    else:
        pipe = oracle_pipeline(wl, procs=procs)
    conn.send({"ready": True, "setup_s": round(time.time() - t0, 1), "flows": pipe.n_flows})
    while True:
        try:
            msg = conn.recv()
        except EOFError:  # the parent went away
            return
        if msg[0] == "check":
            _, cols, verdicts = msg
            t = time.time()
            want = pipe.classify(cols, threads=procs)
            res = compare(verdicts, want)
            res["oracle_s"] = round(time.time() - t, 2)
            conn.send(res)
        elif msg[0] == "churn":  # replay the applied op prefix, then classify against its flows
            t = time.time()
            n = replay_churn(fnp, msg[1])
            t_replay = time.time() - t
            del pipe
            pipe = oracle_pipeline(wl, procs=procs, flows=fnp.dump_flows())
            conn.send({"ops": n, "replay_s": round(t_replay, 1), "rebuild_s": round(time.time() - t - t_replay, 1),
                       "flows": pipe.n_flows})
        elif msg[0] == "baseline":
            _, seconds, chunk = msg
            conn.send(time_baseline(wl, pipe, seconds, chunk, procs))
        else:
            conn.send(None)
            return


def time_baseline(wl, pipe, seconds: float, chunk: int, threads: int) -> dict:
    """The bench `cpu_baseline` object: the C oracle timed on the host cores over chunks of the
    same synthetic workload until `seconds` of wall time have elapsed (setup untimed)."""
    from antrea_amd import workload
    done, elapsed, seed = 0, 0.0, workload.PKT_SEED
    s0 = pipe.stats()
    pipe.classify(workload.gen_packets(wl, 256, seed=seed - 1), threads=threads, count=True)  # warm
    while elapsed < seconds:
        cols = workload.gen_packets(wl, chunk, seed=seed)
        seed += 1
        t = time.perf_counter()
        pipe.classify(cols, threads=threads, count=True)
        elapsed += time.perf_counter() - t
        done += chunk
    s1 = pipe.stats()
    per = {k: round((s1[k] - s0[k]) / max(1, done + 256), 1) for k in s1}
    out = {"value": round(done / elapsed / 1e6, 6), "unit": "Mpps", "cores": threads, "kind": "port",
           "sample": "%d packets of the same synthetic workload (%d-packet chunks), %.1f s, counters on; C restatement "
                     "of OVS 2.17.7 classifier_lookup (TSS + prefix tries + conjunction soft loop) over the %d flows "
                     "the oracle compiler emits" % (done, chunk, elapsed, pipe.n_flows),
           "per_packet": per}
    out.update(host_info())
    env = os.environ.get("OMP_NUM_THREADS")
    out["cores_basis"] = ("OMP_NUM_THREADS=%s: the CPU share the GPU box grants this process (nproc counts the "
                          "whole machine)" % env) if env and env.isdigit() else "the CPUs this process may run on"
    return out


class OracleWorker:
    """CPU oracle in a spawned process (bench.py: parity stamp + CPU baseline)."""

    def __init__(self, config: str, procs: Optional[int] = None, churn: bool = False):
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        self.procs = procs or cpu_threads()
        self.conn, child = ctx.Pipe()
        # not a daemon: the worker forks a pool to convert large flow dumps
        self.p = ctx.Process(target=_serve, args=(child, config, self.procs, churn), daemon=False)
        self.p.start()
        self.info = None
        import atexit
        atexit.register(self.close)  # runs before multiprocessing joins its children

    def _ready(self, timeout=1800):
        if self.info is None:
            import sys
            import time
            t0 = time.time()
            # a progress line every 30 s: a long setup (C2g: ~10 M flows) must not look like a hang
            while not self.conn.poll(30):
                if time.time() - t0 > timeout:
                    raise TimeoutError("oracle worker setup")
                print("[oracle] still setting up (%.0f s)" % (time.time() - t0), file=sys.stderr, flush=True)
            self.info = self.conn.recv()
        return self.info

    def check(self, cols: Dict[str, np.ndarray], verdicts: np.ndarray) -> dict:
        info = self._ready()
        self.conn.send(("check", cols, verdicts))
        res = self.conn.recv()
        res["oracle_setup_s"] = info["setup_s"]
        return res

    def churn(self, ops) -> dict:
        """Replay an op log (replay_churn) in the worker; later checks classify against the result."""
        import sys
        import time
        self._ready()
        self.conn.send(("churn", ops))
        t0 = time.time()
        while not self.conn.poll(20):  # a progress line while the oracle replays (a long log takes minutes)
            print("[oracle] replaying %d ops (%.0f s)" % (len(ops), time.time() - t0), file=sys.stderr, flush=True)
        return self.conn.recv()

    def baseline(self, seconds: float, chunk: int = 4096) -> dict:
        self._ready()
        self.conn.send(("baseline", seconds, chunk))
        return self.conn.recv()

    def close(self):
        if not self.p.is_alive():
            return
        try:
            if self.info is not None:  # idle between requests: ask it to stop
                self.conn.send(("stop",))
                if self.conn.poll(10):
                    self.conn.recv()
        except Exception:
            pass
        self.p.join(timeout=5)
        if self.p.is_alive():
            self.p.terminate()
            self.p.join(timeout=5)
