"""CPU baseline leg of bench.py (TEST / MEASUREMENT INFRASTRUCTURE ONLY, never the product path).

Times the C oracle (oracle/ovs_cls.c: OVS tuple-space-search classifier restated, pthreads) on the
host cores over a bounded sample of the same workload bench.py classifies on the GPU: the same rule
set's realized flows and the same synthetic packet generator, run in chunks until `seconds` of CPU
wall time have elapsed. Reported as kind "port" (a restatement of the reference algorithm, not the
reference binary — OVS is not part of /root/reference).
"""
from __future__ import annotations

import os
import time

import numpy as np

from antrea_amd import workload
from .cls_c import CPipeline


def _threads() -> int:
    n = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    return max(1, min(16, n, os.cpu_count() or 1))


def run(wl, seconds: float = 15.0, flows=None, chunk: int = 4096) -> dict:
    """Returns the bench.py `cpu_baseline` object. `flows` = realized flow text (default: the
    product compiler's dump of wl.rules, pinned against the oracle compiler by the test suite)."""
    if flows is None:
        from antrea_amd import gpc
        clf = gpc.Classifier()
        clf.initialize()
        clf.batch_install_policy_rule_flows(wl.rules)
        flows = clf.dump_flows()
        del clf
    tiers = {r["flow_id"]: int(r.get("tier_priority") or 0) for r in wl.rules}
    t0 = time.time()
    pipe = CPipeline(flows, tiers)
    t_setup = time.time() - t0
    threads = _threads()
    done, elapsed, seed = 0, 0.0, workload.PKT_SEED
    pipe.classify(workload.gen_packets(wl, 256, seed=seed - 1), threads=threads, count=True)  # warm
    while elapsed < seconds:
        cols = workload.gen_packets(wl, chunk, seed=seed)
        cols["len"] = np.full(chunk, 100, np.uint16)
        seed += 1
        t = time.perf_counter()
        pipe.classify(cols, threads=threads, count=True)
        elapsed += time.perf_counter() - t
        done += chunk
    return {"value": round(done / elapsed / 1e6, 6), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": "%d packets of the same synthetic workload (%d-packet chunks), %.1f s, counters on; "
                      "C restatement of OVS classifier_lookup over the %d realized flows (setup %.0f s untimed)"
                      % (done, chunk, elapsed, pipe.n_flows, t_setup)}
