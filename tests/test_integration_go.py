"""The Go binding a maintainer adds (go/pkg/agent/gpuclassify/gpc.go, generated from INTEGRATION.md
by tools/gen_go.py): no Go toolchain here, so these checks are textual -- the file is current with
the document, every C.gpc_* / C.GPC_* symbol it uses is declared in include/gpc.h, and it forwards
every method of the NetworkPolicy half of openflow.Client (SURVEY §8 row b)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "pkg", "agent", "gpuclassify", "gpc.go")


def test_go_file_matches_integration_doc():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_go.py"), "--check"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr


def test_go_uses_only_declared_abi():
    src = open(GO).read()
    hdr = open(os.path.join(ROOT, "include", "gpc.h")).read()
    used = set(re.findall(r"\bC\.((?:gpc|GPC)_\w+)", src))
    assert len(used) > 30
    missing = sorted(u for u in used if not re.search(r"\b%s\b" % re.escape(u), hdr))
    assert not missing, missing


def test_go_forwards_the_np_methods():
    src = open(GO).read()
    methods = ["InstallPolicyRuleFlows", "BatchInstallPolicyRuleFlows", "UninstallPolicyRuleFlows",
               "AddPolicyRuleAddress", "DeletePolicyRuleAddress", "ReassignFlowPriorities",
               "GetPolicyInfoFromConjunction", "NetworkPolicyMetrics", "GetNetworkPolicyFlowKeys",
               "NewDNSPacketInConjunction", "AddAddressToDNSConjunction", "DeleteAddressFromDNSConjunction",
               "InstallServiceGroup", "UninstallServiceGroup", "InstallEndpointFlows", "UninstallEndpointFlows",
               "InstallServiceFlows", "UninstallServiceFlows", "InstallPodFlows"]
    missing = [m for m in methods if not re.search(r"func \(c \*Client\) %s\(" % m, src)]
    assert not missing, missing
    assert src.count("{") == src.count("}") and src.count("(") == src.count(")")
