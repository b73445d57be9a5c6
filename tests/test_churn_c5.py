"""CPU tier of config 5 at full scale: C3 + the seeded op log of tests/golden/make_churn_fixture.py
through the product's C-ABI (delta epochs every 100 ops), the committed image evaluated by the
host emulation of the kernel body (tests/csrc/emu.cpp, the device's core.hpp) == the C oracle's
verdicts over the oracle compiler's replay of the same log (tests/golden/parity_C5.npz), before and
after compaction. The device runs the same in tests/test_gpu_fullscale.py."""
import copy

from antrea_amd import gpc
from oracle import parity
from tests import emu
from tests.golden import make_churn_fixture as cf
from tests.golden import make_parity_fixtures as fx


def test_emulated_product_vs_oracle_after_churn():
    f = cf.load()
    wl, log, cols = cf.inputs()
    assert fx.cols_digest(cols) == str(f["cols_sha256"]) and fx.rules_digest(wl) == str(f["rules_sha256"])
    assert cf.log_digest(log) == str(f["log_sha256"])
    c = gpc.Classifier()
    c.initialize()
    c.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    emu.commit_host(c)
    cf.apply(c, log, on_commit=lambda: emu.commit_host(c))
    st = c.image_stats()
    assert st["n_delta_builds"] > 0 and st["n_tombstones"] > 0
    res = parity.compare(emu.classify(c, cols), f["verdicts"])
    assert res["mismatches"] == 0, res
    emu.commit_host(c, full=True)
    res = parity.compare(emu.classify(c, cols), f["verdicts"])
    assert res["mismatches"] == 0, res
