"""Extracts the NetworkPolicy flow dumps real Antrea agents printed in the reference docs
(`antctl get of -N kube-dns` and `antctl get ovsflows -N test-annp --type ANNP`,
/root/reference/docs/antctl.md:385-400) into tests/golden/antctl_dumps.json (TEST
INFRASTRUCTURE; runs in the build container, where the reference is readable).

    python tests/golden/make_antctl_dumps.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/docs/antctl.md"


def main():
    lines = open(SRC).read().splitlines()
    dumps = []
    for i, l in enumerate(lines):
        m = re.match(r"\$ antctl get (?:of|ovsflows) -N (\S+)", l)
        if not m:
            continue
        flows = []
        for l2 in lines[i + 2:]:  # skip the "FLOW" header
            if not l2.startswith("table="):
                break
            flows.append(l2)
        dumps.append({"policy": m.group(1), "source": "docs/antctl.md:%d-%d" % (i + 1, i + 2 + len(flows)),
                      "flows": flows})
    out = {"note": "ovs-ofctl dump-flows lines of real agents (n_packets / n_bytes included), loaded through "
                   "gpc_load_flows and classified against the oracle", "dumps": dumps}
    with open(os.path.join(HERE, "antctl_dumps.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("%d dumps, %d flows" % (len(dumps), sum(len(d["flows"]) for d in dumps)))


if __name__ == "__main__":
    main()
