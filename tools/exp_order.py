"""Experiment: how much does packet ORDER within the batch change the C3 classify time?

Upper bound for a packet-grouping pre-pass: the batch is reordered OUTSIDE the
timed region (sorted by an address, or grouped so that each XCD's workgroups see one eighth of the
address space) and the two-launch classify step is timed as bench.py does. Prints one JSON line per
ordering. Usage: python tools/exp_order.py [--config C3] [--orders orig,sort_dst,...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def xcd_perm(torch, key, n_xcd=8):
    """Permutation placing packet class c = hash(key) % 8 in the workgroups b with b % 8 == c
    (workgroups are dispatched round-robin over the XCDs); classes truncated to the smallest."""
    h = ((key.to(torch.int64) * 0x9E3779B1) & 0xFFFFFFFF) >> 29
    order = torch.argsort(h, stable=True)
    counts = torch.bincount(h, minlength=n_xcd)
    m = int(counts.min()) // 64 * 64
    starts = torch.cumsum(counts, 0) - counts
    i = torch.arange(m, device=key.device)
    perm = torch.empty(n_xcd * m, dtype=torch.int64, device=key.device)
    for c in range(n_xcd):
        pos = (n_xcd * (i // 64) + c) * 64 + i % 64
        perm[pos] = order[int(starts[c]): int(starts[c]) + m]
    return perm


def _gather(torch, v, perm):
    if v.dtype == torch.uint32:  # no index kernel for uint32: gather the bit pattern as int32
        return v.view(torch.int32)[perm].contiguous().view(torch.uint32)
    return v[perm].contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--group", type=int, default=-1, help="gpc_config.group_packets of the context (-1: off)")
    ap.add_argument("--orders", default="orig,sort_dst,sort_src,xcd_dst16,xcd_src16,xcd_dst24,xcd_src24")
    args = ap.parse_args()
    import torch

    from antrea_amd import gpc, workload
    from antrea_amd.build import build
    build()
    dev = torch.device("cuda", 0)
    wl = workload.CONFIGS[args.config]()
    clf = gpc.Classifier(device=0, group_packets=args.group)
    clf.initialize()
    clf.batch_install_policy_rule_flows(wl.rules)
    if getattr(wl, "services", None):
        workload.install_services(clf, wl)
    clf.commit()
    base = workload.gen_packets_torch(wl, args.packets, device=dev)
    stream = torch.cuda.current_stream(dev)
    for name in args.orders.split(","):
        if name == "orig":
            perm = None
        elif name.startswith("sort_"):  # sort_src / sort_dst, or sort_src16: stable sort on the top 16 bits
            col, bits = name[5:8], int(name[8:] or 32)
            perm = torch.argsort((base[col].to(torch.int64) & 0xFFFFFFFF) >> (32 - bits), stable=True)
        elif name.startswith("tile"):  # tile<T>_<key>: stable sort inside tiles of T packets
            t, rest = name[4:].split("_")
            u = lambda c: base[c].to(torch.int64) & 0xFFFFFFFF
            keys = {"out": lambda: u("out_port") & 255, "s4o4": lambda: ((u("src") >> 28) << 4) | (u("out_port") & 15),
                    "s4d4": lambda: ((u("src") >> 28) << 4) | (u("dst") >> 28),
                    "proto": lambda: (u("proto") & 255), "s6p2": lambda: ((u("src") >> 26) << 2) | (u("proto") & 3)}
            if rest in keys:
                key, bits = keys[rest](), 8
            else:
                col, bits = rest[:3], int(rest[3:])
                key = u(col) >> (32 - bits)
            tile_id = torch.arange(len(key), device=key.device) // int(t)
            perm = torch.argsort((tile_id << bits) | key, stable=True)
        elif name.startswith("gxcd_"):  # gxcd_<col><bits>: global stable sort, XCD x runs the x-th eighth
            col, bits = name[5:8], int(name[8:])
            srt = torch.argsort((base[col].to(torch.int64) & 0xFFFFFFFF) >> (32 - bits), stable=True)
            G = len(srt) // 64
            q, r = G // 8, G % 8
            b = torch.arange(G, device=srt.device)
            x = b % 8
            logical = x * q + torch.minimum(x, torch.full_like(x, r)) + b // 8
            perm = (logical[:, None] * 64 + torch.arange(64, device=srt.device)[None, :]).reshape(-1)
            perm = srt[perm]
        elif name.startswith("xcd_"):
            col, bits = name[4:7], int(name[7:])
            perm = xcd_perm(torch, (base[col].to(torch.int64) & 0xFFFFFFFF) >> (32 - bits))
        else:
            raise SystemExit("unknown order " + name)
        cols = base if perm is None else {k: _gather(torch, v, perm) for k, v in base.items()}
        n = len(cols["src"])
        out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
        soa = gpc.pkt_soa_device(cols)
        for _ in range(3):
            clf.classify_device(soa, n, out.data_ptr(), count=True, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(args.steps):
            clf.classify_device(soa, n, out.data_ptr(), count=True, stream=stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / args.steps
        print(json.dumps({"order": name, "packets": n, "ms_per_step": round(ms, 3),
                          "mpps": round(n / ms / 1e3, 1)}), flush=True)
        del cols, out, soa


if __name__ == "__main__":
    main()
