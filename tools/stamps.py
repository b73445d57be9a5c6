"""Where a classify launch's wave time goes, by code region (diagnostic; GPU box).

Needs the stamp build of the kernel (core.hpp GPC_MARK regions, s_memtime per wave):
    python -c "from antrea_amd import build; build.build(variant='stamps', defines=['GPC_STAMPS'])"
    GPC_LIB=antrea_amd/_build/libgpc_stamps.so python tools/stamps.py --config C3
Prints, per policy-stage launch, the mean cycles per wave charged to each region and its share.
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REGIONS = ["pre", "hard", "drv", "scan", "ver", "tail", "fin", "walk", "post"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from antrea_amd import gpc, workload
    lib = C.CDLL(gpc.LIB_PATH)
    if not hasattr(lib, "gpc_stamps_read"):
        sys.exit("%s is not a stamp build (GPC_STAMPS)" % gpc.LIB_PATH)
    dev = torch.device("cuda", 0)
    wl = workload.CONFIGS[args.config]()
    clf = gpc.Classifier(device=0)
    clf.initialize()
    clf.batch_install_policy_rule_flows(wl.rules)
    if getattr(wl, "services", None):
        workload.install_services(clf, wl)
    clf.commit()
    n = args.packets
    cols = workload.gen_packets_torch(wl, n, seed=workload.PKT_SEED, device=dev)
    soa = gpc.pkt_soa_device(cols)
    out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
    acc = (C.c_ulonglong * 32)()
    clf.classify_device(soa, n, out.data_ptr(), count=True)
    torch.cuda.synchronize()
    lib.gpc_stamps_read(acc, 1)
    for _ in range(args.steps):
        clf.classify_device(soa, n, out.data_ptr(), count=True)
    torch.cuda.synchronize()
    lib.gpc_stamps_read(acc, 0)
    res = {}
    for st, base in (("egress", 0), ("ingress", 16)):
        waves = acc[base + 15]
        if not waves:
            continue
        cyc = [acc[base + i] / waves for i in range(len(REGIONS))]
        tot = sum(cyc)
        res[st] = {"waves": waves, "cycles_per_wave": round(tot), **{r: [round(c), round(100 * c / tot, 1)] for r, c in zip(REGIONS, cyc)}}
        print("%s %-7s cyc/wave %6.0f  " % (args.config, st, tot) + "  ".join("%s %5.0f (%4.1f%%)" % (r, c, 100 * c / tot) for r, c in zip(REGIONS, cyc)))
    print(json.dumps({"config": args.config, "stamps": res}))


if __name__ == "__main__":
    main()
