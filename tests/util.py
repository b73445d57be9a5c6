"""Shared helpers for the test-suite (test vectors -> oracle / product inputs)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def assign_tables(rules):
    """network_policy_test.go:487-501: table by direction and policy type."""
    for r in rules:
        anp = r.get("policy_type", "K8sNetworkPolicy") != "K8sNetworkPolicy"
        if r["direction"] == "Out":
            r.setdefault("table", "AntreaPolicyEgressRule" if anp else "EgressRule")
        else:
            r.setdefault("table", "AntreaPolicyIngressRule" if anp else "IngressRule")
    return rules


def normalize_flows(flows):
    """flowModIgnoreTxIDMatcher (network_policy_test.go:531-570): order-insensitive, conjunction
    actions sorted by conjunction id."""
    out = set()
    for f in flows:
        if "actions=conjunction" not in f:
            out.add(f)
            continue
        prefix, acts = f.split("actions=", 1)
        conjs = acts.replace("),", ")_").split("_")
        conjs.sort(key=lambda c: int(c.replace("conjunction(", "").split(",")[0]))
        out.add(prefix + "actions=" + ",".join(conjs))
    return out
