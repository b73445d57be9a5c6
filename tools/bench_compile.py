"""Control-plane benchmark: BenchmarkBatchInstallPolicyRuleFlows (network_policy_test.go:581-625)
on the product compiler (libgpc, C++) and the oracle compiler (Python). 100 ANNP ingress rules at
priority 100, each From 250 unique + 250 shared addresses, To ofports {1, i}. CPU only.

    python tools/bench_compile.py [--reps 5]
"""
import argparse
import copy
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rules():
    common = ["192.168.0.%d" % i for i in range(250)]
    out = []
    for i in range(100):
        out.append({"direction": "In", "table": "AntreaPolicyIngressRule", "flow_id": i, "priority": 100,
                    "action": "Allow", "policy_type": "AntreaNetworkPolicy", "policy_namespace": "ns1",
                    "policy_name": "np%d" % i, "policy_uid": "id%d" % i, "name": str(i),
                    "from": ["192.169.%d.%d" % (i, j) for j in range(250)] + common,
                    "to": [{"ofport": 1}, {"ofport": i}], "service": None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--oracle", action="store_true", help="also time the Python oracle compiler")
    args = ap.parse_args()
    from antrea_amd import gpc
    rs = rules()
    res = {"benchmark": "BatchInstallPolicyRuleFlows (network_policy_test.go:581-625)", "rules": len(rs)}
    times, marshal = [], []
    for _ in range(args.reps):
        c = gpc.Classifier()
        t0 = time.perf_counter()
        buf = gpc.RuleBuf(copy.deepcopy(rs))  # ctypes marshalling (Python), not part of the library call
        t1 = time.perf_counter()
        rc = c.lib.gpc_batch_install(c.h, buf.arr, buf.n)
        t2 = time.perf_counter()
        assert rc == 0, rc
        times.append(t2 - t1)
        marshal.append(t1 - t0)
        res["flows"] = len(c.dump_flows())
    res["product_ms"] = round(1e3 * min(times), 2)  # gpc_batch_install (C++ compiler) alone
    res["python_marshal_ms"] = round(1e3 * min(marshal), 2)
    if args.oracle:
        from oracle import compiler as oc
        t = time.perf_counter()
        f = oc.FeatureNetworkPolicy()
        f.batch_install_policy_rule_flows(copy.deepcopy(rs))
        res["oracle_ms"] = round(1e3 * (time.perf_counter() - t), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
