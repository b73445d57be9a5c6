"""CPU only: where one packet's image reads go, from the instrumented host build of the kernel body
(tests/csrc/emu.cpp compiles core.hpp with GPC_TOUCH / GPC_STAT hooks). Prints distinct 64-B lines
per packet by source line of core.hpp, plus table lookups, scanned entries and verifications per
packet -- the proxy used to judge image-layout changes before they go to the GPU.

    python tools/emu_lines.py [--config C3] [--packets 20000]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--packets", type=int, default=20000)
    ap.add_argument("--family", type=int, default=4, choices=(4, 6))
    ap.add_argument("--v6-embed", default="96", choices=("96", "multi48"))
    args = ap.parse_args()
    v6 = args.family == 6
    from antrea_amd import gpc, workload
    from tests import emu
    wl = workload.CONFIGS[args.config]()
    c = gpc.Classifier(ipv4=not v6, ipv6=v6)
    c.initialize()
    c.batch_install_policy_rule_flows(workload.to_ipv6(wl, embed=args.v6_embed).rules if v6 else copy.deepcopy(wl.rules))
    if getattr(wl, "services", None):
        workload.install_services(c, wl)
    emu.commit_host(c)
    cols = workload.gen_packets(wl, args.packets, seed=5)
    emu.stats(reset=True)
    emu.site_lines(reset=True)
    if v6:
        emu.classify6(c, workload.packets_to_v6(cols, embed=args.v6_embed))
    else:
        emu.classify(c, cols)
    s, sites = emu.stats(), emu.site_lines()
    n = s[7] or 1
    src = open(os.path.join(os.path.dirname(gpc.HERE), "antrea_amd", "csrc", "core.hpp")).read().split("\n")
    print("%s: %.2f distinct lines / packet; %.2f table lookups, %.2f entries scanned, %.3f verifications "
          "(%.3f failed) per packet" % (args.config, s[6] / n, s[0] / n, s[4] / n, s[3] / n, s[5] / n))
    if v6:
        print("IPv6 codes: %.2f dependent search rounds per packet (src and dst searched together); per address: "
              "%.2f lengths in the regional search, %.3f global searches" % (s[11] / n, s[12] / (2 * n), s[13] / (2 * n)))
        import ctypes as C
        import numpy as np
        lib = emu.load()
        m = min(args.packets, 1 << 20) // 64 * 64
        for col, name in (("gpc_emu_pkt_iter", "src"), ("gpc_emu_pkt_search", "dst")):
            r = np.ctypeslib.as_array((C.c_uint * (1 << 20)).in_dll(lib, col))[:m].copy()
            w = r.reshape(-1, 64).max(axis=1)
            print("  %s: rounds per address mean %.2f, per 64-lane wave (max) mean %.2f, histogram of wave max %s" % (
                name, r.mean(), w.mean(), np.bincount(w).tolist()))
    if not v6:
        import ctypes as C
        import numpy as np
        lib = emu.load()
        m = min(args.packets, 1 << 20) // 64 * 64
        for col, name in (("gpc_emu_pkt_pass", "scan passes"), ("gpc_emu_pkt_iter", "scan iterations"),
                          ("gpc_emu_pkt_search", "verifier search steps"), ("gpc_emu_pkt_verif", "verifications")):
            r = np.ctypeslib.as_array((C.c_uint * (1 << 20)).in_dll(lib, col))[:m].copy()
            w = r.reshape(-1, 64).max(axis=1)
            print("  %-22s per packet mean %.2f, per 64-lane wave (max) mean %.2f" % (name, r.mean(), w.mean()))
    for line, v in sorted(sites.items(), key=lambda kv: -kv[1]):
        if v / n >= 0.01:
            print("  core.hpp:%-5d %6.2f  %s" % (line, v / n, src[line - 1].strip()[:70]))


if __name__ == "__main__":
    main()
