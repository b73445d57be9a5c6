"""bench.py roofline arithmetic (CPU): the dominant launch kind, its counter bytes per launch over
its HIP-event time, the step figures beside it, and the sanity bound (frac <= 1)."""
import pytest

import bench


def _pmc():
    k1 = "classify_kernel<false, false, 1, false, false>"
    k2 = "classify_kernel<false, false, 2, false, false>"
    passes = [{"by_kernel": {k1: {"FETCH_SIZE": 1000.0}, k2: {"FETCH_SIZE": 3000.0}}},
              {"by_kernel": {k1: {"WRITE_SIZE": 500.0, "TCC_HIT_sum": 9.0, "TCC_MISS_sum": 1.0},
                             k2: {"WRITE_SIZE": 200.0, "TCC_HIT_sum": 8.0, "TCC_MISS_sum": 2.0}}}]
    return {"FETCH_SIZE": 4000.0, "WRITE_SIZE": 700.0, "TCC_HIT_sum": 17.0, "TCC_MISS_sum": 3.0, "_passes": passes}


def test_dominant_kernel_roofline():
    launches = {"classify_egress": {"mean_ms": 0.001, "per_step": 1.0},
                "classify_ingress": {"mean_ms": 0.002, "per_step": 1.0}}
    rl = bench._roofline(_pmc(), 0.003, 1000, 17, 16, 10.0, launches)
    assert rl["kernel"] == "classify_ingress"
    tr = (2 * 3000.0 + 200.0) * 1024
    assert rl["traffic"] == int(tr)
    assert rl["achieved"] == pytest.approx(round(tr / 0.002e-3 / 1e9, 1))
    assert rl["frac"] == pytest.approx(rl["achieved"] / 8000.0, abs=1e-4)
    assert rl["frac_without_fetch_x2"] < rl["frac"]
    step = rl["step"]
    assert step["traffic"] == int((2 * 4000.0 + 700.0) * 1024)
    assert step["l2_hit_rate"] == pytest.approx(0.85)
    assert rl["kernels"]["classify_egress"]["bytes_per_packet"] == pytest.approx((2 * 1000 + 500) * 1024 / 1000, abs=0.1)
    assert rl["algorithmic"]["frac_if_uncached"] > 0


def test_roofline_rejects_above_peak():
    launches = {"classify_ingress": {"mean_ms": 1e-9, "per_step": 1.0}}
    with pytest.raises(RuntimeError):
        bench._roofline(_pmc(), 0.003, 1000, 17, 16, None, launches)
