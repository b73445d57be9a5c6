"""Generates tests/golden/parity_<config>.npz: the C oracle's verdicts and per-rule metrics for
full-size workloads (TEST INFRASTRUCTURE; run here, on the CPU, never on the GPU box).

    python tests/golden/make_parity_fixtures.py [C1 C2 C3 C4 ...]

For each config: the workload (antrea_amd.workload, rule seed 0xA1E47) compiled by the ORACLE
compiler (oracle/compiler.py), loaded into the C restatement of the OVS classifier
(oracle/ovs_cls.c), which classifies N packets of the seeded generator (seed below) with counters
on. Stored: the verdicts (n x 2 records of 8 B, gpc_verdict layout), the metrics
{conj: (packets, bytes, sessions)} as NetworkPolicyMetrics parses the Metric-table dump, a SHA-256
of the packet columns and of the rule list (so a generator change is detected instead of silently
comparing different inputs), and for C4 the Service stage's LB result words of every packet (the C
oracle runs the AntreaProxy stage, ovs_cls.c service_stage, over the ServiceLB / EndpointDNAT flows
and groups the product realizes -- text pinned by the reference's client_test.go goldens). `mask`
(kept for the loaders) selects every packet.
"""
from __future__ import annotations

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

SPECS = {  # config -> (packets, packet seed); "x": the workload with every optional packet column set
    "C1": (100_000, 0xF1C1),
    "C2": (100_000, 0xF1C2),
    "C3": (100_000, 0xF1C3),
    "C4": (100_000, 0xF1C4),
    "C3x": (100_000, 0xF1C5),
    "C2g": (100_000, 0xF1C6),  # C2 with AddressGroups of 10k Pod IPs (BASELINE configs[1] as worded)
}
COLS = ("src", "dst", "sport", "dport", "proto", "out_port", "len")
OPT_COLS = ("in_port", "tun_id", "ct_src", "ct_dst", "ct_state", "dest", "ct_mark", "svc_group")


def optional_columns(cols, seed):
    """Every optional column of gpc_pkt_soa, seeded: conntrack states (new / est / rel / reply, the
    64990 skip flows and the DNS +rpl flow), pre-NAT addresses, IngressSecurityClassifier
    destinations (Pod / gateway / tunnel / uplink) and the hairpin ct_mark, in_port, tun_id, reg7."""
    rng = np.random.default_rng(seed)
    n = len(cols["src"])
    out = dict(cols)
    out["in_port"] = rng.integers(0, 200, n).astype(np.uint32)
    out["tun_id"] = rng.integers(0, 4, n).astype(np.uint32)
    out["ct_src"] = np.where(rng.random(n) < 0.9, cols["src"], rng.integers(0, 1 << 32, n)).astype(np.uint32)
    out["ct_dst"] = np.where(rng.random(n) < 0.9, cols["dst"], rng.integers(0, 1 << 32, n)).astype(np.uint32)
    out["ct_state"] = rng.choice([0x21, 0x22, 0x24, 0x2a, 0x29], size=n, p=[0.75, 0.1, 0.05, 0.05, 0.05]).astype(np.uint8)
    out["dest"] = rng.choice(4, size=n, p=[0.85, 0.05, 0.05, 0.05]).astype(np.uint8)
    out["ct_mark"] = np.where(rng.random(n) < 0.05, 0x40, 0).astype(np.uint8)
    out["svc_group"] = np.where(rng.random(n) < 0.1, rng.integers(1, 50, n), 0).astype(np.uint32)
    return out


def cols_digest(cols) -> str:
    h = hashlib.sha256()
    for k in COLS + tuple(c for c in OPT_COLS if c in cols):
        h.update(k.encode())
        h.update(np.ascontiguousarray(cols[k]).tobytes())
    return h.hexdigest()


def rules_digest(wl) -> str:
    return hashlib.sha256(json.dumps(wl.rules, sort_keys=True, default=str).encode()).hexdigest()


def path(config: str) -> str:
    return os.path.join(HERE, "parity_%s.npz" % config)


def packets(config: str, wl=None):
    n, seed = SPECS[config]
    wl = wl or workload.CONFIGS[config[:-1] if config.endswith("x") else config]()
    cols = workload.gen_packets(wl, n, seed=seed)
    return wl, optional_columns(cols, seed) if config.endswith("x") else cols


def make(config: str):
    t0 = time.time()
    wl, cols = packets(config)
    pipe = parity.oracle_pipeline(wl)
    t1 = time.time()
    want, lb = pipe.classify(cols, threads=parity.cpu_threads(), count=True, lb=True)
    t2 = time.time()
    mask = np.ones(len(cols["src"]), bool)
    m = parity.oracle_metrics(pipe)
    conj = np.array(sorted(m), np.uint32)
    met = np.array([m[int(c)] for c in conj], np.uint64).reshape(-1, 3)
    extra = {"lb": lb} if getattr(wl, "services", None) else {}
    np.savez_compressed(path(config), verdicts=np.ascontiguousarray(want).view(np.uint32).reshape(-1, 4),
                        metric_conj=conj, metric_val=met, mask=mask, cols_sha256=cols_digest(cols),
                        rules_sha256=rules_digest(wl), n_flows=pipe.n_flows, **extra)
    print("%s: %d packets, %d flows, oracle setup %.0f s, classify %.1f s, %d metric rules%s"
          % (config, len(cols["src"]), pipe.n_flows, t1 - t0, t2 - t1, len(conj),
             ", %d Service hits" % int((lb[:, 1] >> 16 != 0).sum()) if extra else ""))


def load(config: str) -> dict:
    with np.load(path(config), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["verdicts"] = np.ascontiguousarray(d["verdicts"]).view(parity.VERDICT_NP).reshape(-1, 2)
    d["metrics"] = {int(c): tuple(int(x) for x in v) for c, v in zip(d["metric_conj"], d["metric_val"])}
    return d


if __name__ == "__main__":
    for c in sys.argv[1:] or sorted(SPECS):
        make(c)
