"""Extract + check the e2e reachability expectations and write `e2e_reachability.json`.

Run in the build container (reads /root/reference as text; never on the GPU box):

    python -m tests.golden.make_e2e_reachability

For every step of `e2e_cases.CASES` it parses the reference's own `reachability.go` calls
(NewReachability / Expect* on the named variable, inside the cited line range of the cited test
function) and the NPEvaluation chain, and fails unless they equal the hand transcription. The
networkpolicy_test.go cases are single probes: their `runNetcatCommandFromTestPod` / `npCheck`
conditions are counted instead (err != nil -> must connect, err == nil / wantErr -> must not).
The fixture then holds the transcription plus each step's full expected matrix. It copies no
reference source: only the expectations (data) and the line numbers they came from.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.e2e_cases import CASES  # noqa: E402
from tests import e2e_model as em  # noqa: E402

REF = os.environ.get("ANTREA_REF", "/root/reference")
OUT = os.path.join(HERE, "e2e_reachability.json")

METHODS = {"Expect": "expect", "ExpectSelf": "self", "ExpectAllIngress": "all_ingress", "ExpectAllEgress": "all_egress",
           "ExpectAllSelfNamespace": "all_self_ns", "ExpectSelfNamespace": "self_ns",
           "ExpectIngressFromNamespace": "ingress_from_ns", "ExpectEgressToNamespace": "egress_to_ns",
           "ExpectNamespaceIngressFromNamespace": "ns_ingress_from_ns",
           "ExpectNamespaceEgressToNamespace": "ns_egress_to_ns"}
EVAL_ACT = {"NPEvalAllow": "Allow", "NPEvalDrop": "Drop", "NPEvalIsolate": "Isolate", "NPEvalReject": "Reject"}


def _args(text):
    """Split a Go call's argument list at top-level commas."""
    out, depth, cur = [], 0, ""
    for ch in text:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _pod(a):
    m = re.fullmatch(r'getPod\("([\w-]+)", "([\w-]+)"\)', a)
    if m:
        return "%s/%s" % m.groups()
    m = re.fullmatch(r'Pod\(getNS\("([\w-]+)"\)\s*\+\s*"/([\w-]+)"\)', a)
    if m:
        return "%s/%s" % m.groups()
    raise ValueError("pod expression %r" % a)


def _ns(a):
    m = re.fullmatch(r'getNS\("([\w-]+)"\)', a)
    if not m:
        raise ValueError("namespace expression %r" % a)
    return m.group(1)


def _call(line, var):
    m = re.search(r"\b%s\s*:?=\s*NewReachability\(allPods,\s*(\w+)\)" % re.escape(var), line)
    if m:
        return ["new", m.group(1)]
    m = re.search(r"\b%s\.(\w+)\((.*)\)\s*$" % re.escape(var), line.strip())
    if not m:
        return None
    meth, args = m.group(1), _args(m.group(2))
    kind = METHODS.get(meth)
    if kind is None:
        return None
    mark = args[-1]
    if kind == "expect":
        return [kind, _pod(args[0]), _pod(args[1]), mark]
    if kind in ("self", "all_self_ns"):
        return [kind, mark]
    if kind in ("all_ingress", "all_egress"):
        return [kind, _pod(args[0]), mark]
    if kind == "self_ns":
        return [kind, _ns(args[0]), mark]
    if kind in ("ingress_from_ns", "egress_to_ns"):
        return [kind, _pod(args[0]), _ns(args[1]), mark]
    return [kind, _ns(args[0]), _ns(args[1]), mark]


def _function(lines, name):
    start = next(i for i, l in enumerate(lines) if re.match(r"func %s\(" % re.escape(name), l))
    end = next((i for i in range(start + 1, len(lines)) if lines[i].startswith("func ")), len(lines))
    return start, end


def _builder_names(body):
    names = {"defaultDenyKNPName": "default-deny-namespace"}
    for m in re.finditer(r'(\w+)\s*:?=\s*\w+\.SetName\((?:getNS\("[\w-]+"\),\s*)?"([^"]+)"\)', body):
        names[m.group(1) + ".Name"] = m.group(2)
    return names


def _eval_calls(lines, lo, hi, var, names):
    text = " ".join(l.strip() for l in lines[lo - 1:hi])
    m = re.search(r"\b%s\s*:?=\s*NewNPEvaluation\(allPods\)\.(.*)" % re.escape(var), text)
    if not m:
        raise ValueError("no NewNPEvaluation for %s" % var)
    out = []
    for c in re.finditer(r"(Expect|ExpectNone)\(((?:[^()]|\([^()]*\))*)\)", m.group(1)):
        a = _args(c.group(2))
        if c.group(1) == "ExpectNone":
            out.append([_pod(a[0]), _pod(a[1]), "<NONE>", "<NONE>"])
        else:
            out.append([_pod(a[0]), _pod(a[1]), names[a[2]], EVAL_ACT[a[3]]])
    return out


def _netcat_marks(lines, lo, hi):
    marks = []
    for l in lines[lo - 1:hi]:
        if "runNetcatCommandFromTestPod" in l and "err != nil" in l:
            marks.append("Connected")
        elif "runNetcatCommandFromTestPod" in l and "err == nil" in l:
            marks.append("Dropped")
        else:
            m = re.search(r"npCheck\(.*,\s*(true|false)\)\s*$", l.strip())
            if m:
                marks.append("Dropped" if m.group(1) == "true" else "Connected")
    return sorted(marks)


def verify(cases):
    files = {}
    checked = 0
    for c in cases:
        path = os.path.join(REF, c["go_file"])
        if path not in files:
            with open(path) as f:
                files[path] = f.read().split("\n")
        lines = files[path]
        fs, fe = _function(lines, c["go_func"])
        names = _builder_names("\n".join(lines[fs:fe]))
        for st in c["steps"]:
            var, lo, hi = st["src"]
            assert fs < lo <= hi <= fe, (c["name"], st["name"], "range outside %s" % c["go_func"])
            if c["go_file"].endswith("networkpolicy_test.go"):
                want = sorted(op[-1] for op in st["reach"])
                got = _netcat_marks(lines, lo, hi)
                assert got == want, (c["name"], st["name"], got, want)
            else:
                got = [op for op in (_call(l, var) for l in lines[lo - 1:hi]) if op]
                assert got == st["reach"], (c["name"], st["name"], got, st["reach"])
            if st["eval"]:
                ev, elo, ehi = st["eval_src"]
                assert fs < elo <= ehi <= fe
                got = _eval_calls(lines, elo, ehi, ev, names)
                assert got == st["eval"], (c["name"], st["name"], got, st["eval"])
            checked += 1
    return checked, {os.path.relpath(p, REF): hashlib.sha256("\n".join(l).encode()).hexdigest() for p, l in files.items()}


def universe(c):
    u = c["universe"]
    if u == "xyz":
        return em.Universe({"x": {}, "y": {}, "z": {}})
    if "namespaces" in u:
        return em.Universe(u["namespaces"], [tuple(p) for p in u["pods"]], family=u.get("family", 4))
    return em.Universe(u)


def main():
    checked, digests = verify(CASES)
    out = {"about": "e2e reachability expectations of the reference (see make_e2e_reachability.py)",
           "reference_files": digests, "steps_checked": checked, "cases": []}
    for c in CASES:
        u = universe(c)
        cc = dict(c)
        cc["steps"] = []
        for st in c["steps"]:
            m = em.expected_matrix(u, st["reach"])
            s2 = dict(st)
            s2["expected"] = sorted([a, b, v] for (a, b), v in m.items())
            cc["steps"].append(s2)
        out["cases"].append(cc)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote %s: %d cases, %d steps checked against the reference" % (OUT, len(CASES), checked))


if __name__ == "__main__":
    main()
