"""Host-side pieces of bench.py that run without a GPU (C5 control loop)."""
import threading
import time

import bench
from antrea_amd import workload


class _Stub:
    def __init__(self):
        self.ops = 0
        self.commits = 0

    def add_policy_rule_address(self, *a):
        self.ops += 1

    def delete_policy_rule_address(self, *a):
        self.ops += 1

    def commit(self):
        self.commits += 1
        time.sleep(0.002)


def test_churn_loop_paces_ops_and_records_latency():
    wl = workload.config1()
    stub, rec, stop = _Stub(), [], threading.Event()
    ops = bench._ChurnOps(stub, wl, seed=1)
    th = threading.Thread(target=bench._churn_loop, args=(ops, 5000.0, 2000, stop, rec))
    th.start()
    time.sleep(0.5)
    stop.set()
    th.join()
    n = sum(r[0] for r in rec)
    assert n == stub.ops == ops.issued and len(rec) == stub.commits
    ops = n
    assert 1500 <= ops <= 3500  # ~5000 ops/s for 0.5 s
    assert all(len(r[2]) == r[0] and (r[2] >= 0).all() for r in rec)


def test_churn_ops_same_seed_same_stream():
    """C5 at N>1: every rank draws the same op sequence, whatever its batching."""
    wl = workload.config1()

    class Rec(_Stub):
        def __init__(self):
            super().__init__()
            self.seq = []

        def add_policy_rule_address(self, *a):
            self.seq.append(("add",) + tuple(map(str, a)))

        def delete_policy_rule_address(self, *a):
            self.seq.append(("del",) + tuple(map(str, a)))

    a, b = Rec(), Rec()
    oa, ob = bench._ChurnOps(a, wl, seed=1234), bench._ChurnOps(b, wl, seed=1234)
    for _ in range(50):
        oa.apply(7)
    for _ in range(7):
        ob.apply(50)
    assert a.seq == b.seq[:350] and len(a.seq) == 350


def test_grouping_label_from_launches():
    """The bench line's packet_grouping field names what ran (no GPU: launch names only)."""
    import bench
    from antrea_amd import gpc
    st = {"group_key": gpc.GROUP_KEY_ADDR}
    assert bench._grouping_label(st, {"classify_egress": {}}, False) == "off"
    lab = bench._grouping_label(st, {"group_tiles": {}, "unpermute": {}}, False)
    assert lab.startswith("key: top 8 bits of nw_src") and lab.endswith("results un-permuted")
    assert "IPv6 code columns" in bench._grouping_label(st, {"group_tiles": {}}, True)
    assert "scan-length" in bench._grouping_label({"group_key": gpc.GROUP_KEY_SCAN}, {"group_tiles": {}}, False)
