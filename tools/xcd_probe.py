"""GPU experiment (no product code): would a stage launch gain if each XCD's L2 only ever saw 1/8 of
the stage's driver index? The same C3 batch is classified in three orders: as generated, and
permuted so that the blocks sharing an XCD (blocks b with equal b % 8 under round-robin dispatch,
MI355X_MICROARCH.md "Workgroup dispatch") get only packets whose driver band key -- egress: dst /12,
ingress: src /12 (C3's composite tables are keyed at band 0, /12) -- hashes to that residue. The permutation is
made with torch before the timed region; verdicts do not depend on the order.

    python tools/xcd_probe.py [--packets 67108864] [--steps 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--block", type=int, default=64)
    args = ap.parse_args()
    import torch
    from antrea_amd import gpc, workload
    dev = torch.device("cuda:0")
    wl = workload.CONFIGS[args.config]()
    clf = gpc.Classifier(device=0)
    clf.initialize()
    clf.batch_install_policy_rule_flows(wl.rules)
    clf.commit()
    cols = workload.gen_packets_torch(wl, args.packets, seed=77, device=dev)
    B = args.block

    def i64(t):
        return t.view(torch.int32).to(torch.int64) & 0xFFFFFFFF if t.dtype == torch.uint32 else t.to(torch.int64)

    def part(t):  # core.hpp cbucket_class of the band-0 key (/12): the slice of the index it touches
        return ((((i64(t) >> 20) * 0x9E3779B1) & 0xFFFFFFFF) >> 29)

    def order(p):
        srt = torch.argsort(p, stable=True)
        sizes = torch.bincount(p, minlength=8)
        chunks = int(sizes.min().item()) // B
        starts = torch.cumsum(sizes, 0) - sizes
        # block b = 8 * j + r takes packets [starts[r] + j*B, +B) of the sorted order
        j = torch.arange(chunks, device=dev).view(chunks, 1, 1)
        r = torch.arange(8, device=dev).view(1, 8, 1)
        k = torch.arange(B, device=dev).view(1, 1, B)
        return srt[(starts.view(1, 8, 1) + j * B + k).reshape(-1)], chunks * 8 * B

    def take(idx):
        return {k: (v.view(torch.int32)[idx].view(v.dtype) if v.dtype == torch.uint32 else v[idx]).contiguous()
                for k, v in cols.items()}

    # control: a batch of class-0 packets only (every XCD touches the same 1/8 slice)
    def only(p, r=0):
        idx = (p == r).nonzero().squeeze(1)
        return idx[: idx.numel() // (8 * B) * (8 * B)]

    pe, ne = order(part(cols["dst"]))
    pi, ni = order(part(cols["src"]))
    N = args.packets
    cases = [("generated", torch.arange(N, device=dev)), ("egress-key XCD partition", pe), ("ingress-key XCD partition", pi),
             ("egress-key class 0 only", only(part(cols["dst"]))), ("ingress-key class 0 only", only(part(cols["src"])))]
    out = torch.empty(2 * N * 8, dtype=torch.uint8, device=dev)
    ref = None
    for name, idx in cases:
        n = idx.numel()
        c = take(idx)
        soa = gpc.pkt_soa_device(c)
        for _ in range(3):
            clf.classify_device(soa, n, out.data_ptr(), count=True)
        torch.cuda.synchronize()
        clf.launch_times()
        clf.set_launch_timing(args.steps)
        for _ in range(args.steps):
            clf.classify_device(soa, n, out.data_ptr(), count=True)
        torch.cuda.synchronize()
        t = clf.launch_times()
        v = out[:16 * n].view(n, 16).cpu()
        # same verdicts as the generated order, packet by packet
        same = "-" if ref is None else bool(torch.equal(v, ref[idx.cpu()]))
        if ref is None:
            ref = v
        print("%-26s n=%d ms per 2^26 packets %s same verdicts: %s" % (
            name, n, {k: round(x["mean_ms"] * (1 << 26) / n, 3) for k, x in t.items()}, same), flush=True)
        del c, soa


if __name__ == "__main__":
    main()
