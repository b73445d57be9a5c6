"""GPU tier: the reference's e2e verdict tables on the device (see tests/test_e2e_reachability.py).

Every step of every case runs the model reconciler against the product, publishes the epoch with
gpc_commit (steps after the first go through delta epochs: Add/DeletePolicyRuleAddress,
Uninstall / Install), classifies one packet per (Pod pair, port) with gpc_classify (gpc_classify6
for the IPv6 cases) and checks: the reference's expected mark for every pair, verdicts equal to
the oracle's bit for bit, and every NPEvaluation assertion. The last step is repeated after
gpc_compact (full rebuild)."""
import pytest

from tests import e2e_run
from tests.test_e2e_reachability import CASES, _check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


def test_e2e_reachability_on_device():
    n_pairs = 0
    for case in CASES:
        n_pairs += _check(e2e_run.run_case(case, backend="device"))
    assert n_pairs >= 5000
