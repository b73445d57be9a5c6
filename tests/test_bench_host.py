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
    th = threading.Thread(target=bench._churn_loop, args=(stub, wl, 5000.0, 2000, stop, rec, 1))
    th.start()
    time.sleep(0.5)
    stop.set()
    th.join()
    ops = sum(r[0] for r in rec)
    assert ops == stub.ops and len(rec) == stub.commits
    assert 1500 <= ops <= 3500  # ~5000 ops/s for 0.5 s
    assert all(len(r[2]) == r[0] and (r[2] >= 0).all() for r in rec)
