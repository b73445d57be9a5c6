"""C5 control-plane cost on this host (diagnostic): per-op time of bench.py's address-op stream
against C3, alone and while another thread keeps the device classifying, and per-commit time."""
import copy
import sys
import threading
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from antrea_amd import gpc, workload
    wl = workload.CONFIGS["C3"]()
    clf = gpc.Classifier(device=0)
    clf.initialize()
    clf.batch_install_policy_rule_flows(copy.deepcopy(wl.rules))
    clf.commit()
    ops = bench._ChurnOps(clf, wl, seed=7)
    t = time.perf_counter()
    ops.apply(20000)
    t_ops = time.perf_counter() - t
    t = time.perf_counter()
    clf.commit()
    t_commit = time.perf_counter() - t
    print("alone: %.1f us/op, commit of 20000 ops %.1f ms" % (t_ops / 20000 * 1e6, t_commit * 1e3), flush=True)
    n = 1 << 24
    dev = torch.device("cuda", 0)
    cols = workload.gen_packets_torch(wl, n, seed=1, device=dev)
    soa = gpc.pkt_soa_device(cols)
    out = torch.empty(2 * n * 8, dtype=torch.uint8, device=dev)
    stop = threading.Event()

    def run():
        s = torch.cuda.current_stream(dev).cuda_stream
        while not stop.is_set():
            clf.classify_device(soa, n, out.data_ptr(), count=True, stream=s)
        torch.cuda.synchronize(dev)

    th = threading.Thread(target=run)
    th.start()
    time.sleep(0.5)
    for k in range(3):
        t = time.perf_counter()
        ops.apply(5000)
        t_ops = time.perf_counter() - t
        t = time.perf_counter()
        clf.commit()
        t_commit = time.perf_counter() - t
        print("beside classification: %.1f us/op, commit of 5000 ops %.1f ms" % (t_ops / 5000 * 1e6, t_commit * 1e3),
              flush=True)
    stop.set()
    th.join()
    print(clf.image_stats()["n_overlay_rules"], "overlay rules")


if __name__ == "__main__":
    main()
