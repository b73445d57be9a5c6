"""Flow-text ingest of real agents' dumps: the NetworkPolicy flows Antrea agents
printed in the reference docs (`antctl get of -N kube-dns`, `antctl get ovsflows -N test-annp
--type ANNP`; docs/antctl.md:383-400, extracted by tests/golden/make_antctl_dumps.py, n_packets /
n_bytes fields included) are loaded with gpc_load_flows and classified; the verdicts must equal the
oracle's walk of the same text. CPU tier through the host emulation, GPU tier on the device."""
import numpy as np
import pytest

from antrea_amd import gpc
from oracle import ovs_cls
from tests import emu
from tests.test_emu_parity import _cmp
from tests.util import load_golden

DUMPS = {d["policy"]: d["flows"] for d in load_golden("antctl_dumps.json")["dumps"]}
SETS = {"kube-dns": DUMPS["kube-dns"], "test-annp": DUMPS["test-annp"],
        "both": DUMPS["kube-dns"] + DUMPS["test-annp"]}


def _packets(n=4000, seed=3):
    rng = np.random.default_rng(seed)
    srcs = np.array([0x0A140108, 0x0A140208, 0x0A140308, 0xAC640107], np.uint32)  # 10.20.1.8, 10.20.2.8, ...
    cols = {"src": np.where(rng.random(n) < 0.7, rng.choice(srcs, n), rng.integers(0, 1 << 32, n)).astype(np.uint32),
            "dst": rng.integers(0, 1 << 32, n).astype(np.uint32),
            "sport": rng.integers(1024, 65536, n).astype(np.uint16),
            "dport": rng.choice([53, 443, 9153, 80, 8080], n).astype(np.uint16),
            "proto": rng.choice([6, 17, 1], n, p=[0.6, 0.3, 0.1]).astype(np.uint8),
            "out_port": rng.choice([3, 5, 7], n).astype(np.uint32),
            "len": rng.integers(64, 1500, n).astype(np.uint16)}
    return cols


def _oracle(flows, cols):
    pipe = ovs_cls.Pipeline(flows)
    n = len(cols["src"])
    out = np.zeros((n, 2), dtype=gpc.VERDICT_DTYPE)
    for i in range(n):
        e, g = pipe.classify({k: int(v[i]) for k, v in cols.items()})
        for j, v in enumerate((e, g)):
            out[i, j] = (v[1], v[0], v[2], v[3], v[4])
    return out


def _loaded(flows):
    c = gpc.Classifier()
    loaded, skipped = c.load_flows(flows)
    assert loaded == len(flows) and skipped == 0
    return c


@pytest.mark.parametrize("name", sorted(SETS))
def test_real_dump_emu_vs_oracle(name):
    flows = SETS[name]
    cols = _packets()
    c = _loaded(flows)
    emu.commit_host(c)
    want = _oracle(flows, cols)
    _cmp(emu.classify(c, cols), want, cols)
    acts = set(int(a) for a in want[:, 1]["action"])
    assert 2 in acts or 3 in acts, acts  # the dump's rules decide some packets


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SETS))
def test_real_dump_device_vs_oracle(name):
    from antrea_amd.build import build
    build()
    flows = SETS[name]
    cols = _packets(20000, seed=4)
    c = _loaded(flows)
    c.commit()
    got = c.classify_host(cols)
    _cmp(got, _oracle(flows, cols), cols)
