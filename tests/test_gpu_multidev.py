"""GPU tier: one control plane over several device slots (gpc_create_multi) next to an ordinary
one-device context, both driven through the same delta stream.

The box has one GPU, so the multi-device context gets slots [0, 0]: two independent copies of
every epoch (images, journal pools, counters, grouping scratch) on one device -- the same code
path as [0..7] on a node, minus the device switch."""
import copy

import numpy as np
import pytest

from antrea_amd import gpc, workload
from tests import emu
from tests.test_emu_parity import _cmp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _built():
    from antrea_amd.build import build
    build()
    import torch
    assert torch.cuda.is_available(), "GPU tier needs a HIP device"


def _ip(v):
    return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)


@pytest.mark.parametrize("group", [-1, 1], ids=["plain", "grouped"])
def test_two_slots_and_two_contexts_same_delta_stream(group):
    wl = workload.config1(seed=41)
    n = 30000
    cols = workload.gen_packets(wl, n, seed=41)
    rng = np.random.default_rng(41)
    multi = gpc.Classifier(devices=[0, 0], group_packets=group)
    single = gpc.Classifier(device=0, group_packets=group)
    assert multi.n_devices == 2 and single.n_devices == 1
    rules = copy.deepcopy(wl.rules)
    for c in (multi, single):
        c.initialize()
        c.batch_install_policy_rule_flows(copy.deepcopy(rules))
        c.commit()
    by_id = {r["flow_id"]: r for r in rules}
    ids = sorted(by_id)
    for step in range(16):
        rid = int(rng.choice(ids))
        r = by_id[rid]
        side = "src" if r.get("from") else "dst"
        lst = r.get("from") if side == "src" else r.get("to")
        if step % 6 == 5:
            for c in (multi, single):
                c.uninstall_policy_rule_flows(rid)
                c.commit()
                c.install_policy_rule_flows(copy.deepcopy(r))
        elif lst is not None:
            addrs = [_ip(int(cols[side][i])) for i in rng.choice(n, size=6, replace=False)]
            for c in (multi, single):
                c.add_policy_rule_address(rid, side, addrs, r.get("priority"))
            lst.extend(addrs)
        for c in (multi, single):
            c.commit()
        if step % 5 == 0:  # every slot classifies on the epoch just published
            a = multi.classify_host(cols, slot=0)
            b = multi.classify_host(cols, slot=1)
            assert np.array_equal(a, b), step
            assert multi.stream_epoch() == multi.image_stats()["epoch"]
    sm, ss = multi.image_stats(), single.image_stats()
    assert sm["epoch"] == ss["epoch"] and sm["n_delta_builds"] == ss["n_delta_builds"] >= 12
    assert sm["n_overlay_rules"] == ss["n_overlay_rules"] > 0 and sm["n_ext_rules"] == ss["n_ext_rules"]
    multi.reset_counters()
    single.reset_counters()
    multi.set_launch_timing(8)
    v0 = multi.classify_host(cols, count=True, slot=0)
    v1 = multi.classify_host(cols, count=True, slot=1)
    vs = single.classify_host(cols, count=True)
    want = emu.classify(single, cols)
    _cmp(vs, want, cols)
    assert np.array_equal(v0, vs) and np.array_equal(v1, vs)
    lt = multi.launch_times()
    multi.set_launch_timing(0)
    assert lt and sum(t["launches"] for t in lt.values()) >= 4  # both slots' launches were timed
    # per-slot counters each equal the single context's; gpc_metrics sums the slots in-process
    ms = {k: v for k, v in single.network_policy_metrics().items() if any(v)}
    mm = {k: v for k, v in multi.network_policy_metrics().items() if any(v)}
    assert ms and mm == {k: tuple(2 * x for x in v) for k, v in ms.items()}
    p0, slots0 = multi.counters(slot=0)
    p1, slots1 = multi.counters(slot=1)
    assert p0 and p1 and p0 != p1 and slots0 == slots1
    # compaction publishes the new base on both slots
    multi.compact()
    single.compact()
    assert multi.image_stats()["n_overlay_rules"] == 0
    assert np.array_equal(multi.classify_host(cols, slot=1), vs)
    assert np.array_equal(multi.classify_host(cols, slot=0), vs)
    multi.close()
    single.close()


def test_slot_out_of_range_is_einval():
    c = gpc.Classifier(devices=[0])
    c.initialize()
    c.commit()
    cols = workload.gen_packets(workload.config1(seed=1), 16, seed=1)
    with pytest.raises(gpc.GpcError) as e:
        c.classify_host(cols, slot=1)
    assert e.value.code == gpc.GPC_EINVAL
    c.close()


def test_bench_multidev_two_slots():
    """bench.py --multidev: one process, gpc_create_multi over two slots of the
    box's one GPU ([0, 0]), one stream and host thread per slot, the standard JSON line, verdicts of
    both slots checked against the C oracle on a sample, counters summed over the slots."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--multidev", "2", "--multidev-devices", "0,0", "--config",
           "C1", "--steps", "3", "--warmup", "1", "--packets", str(1 << 20), "--no-traffic", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["slots"] == 2 and line["config"]["devices"] == [0, 0]
    assert line["value"] > 0 and len(line["slot_kernel_ms"]) == 2
    assert line["parity"]["checked"] > 0 and line["parity"]["mismatches"] == 0, line["parity"]
    assert line["metrics_rules_nonzero"] > 0
