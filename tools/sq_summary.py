"""Summarise rocprofv3 SQ counter CSVs (tools/sq_profile.sh output) per kernel: per-wave instruction
counts and wave-cycle shares.

    python tools/sq_summary.py gpurun_out/TAG [more dirs]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"classify_kernel<(\w+), (\w+), (\d), (\w+)>", name)
    if m:
        return "classify<d=%s,s=%s,st=%s,sort=%s>" % (m.group(1)[0], m.group(2)[0], m.group(3), m.group(4)[0])
    return re.sub(r"\(.*", "", name).replace("void gpc::", "")[:40]


def load(d):
    acc = defaultdict(lambda: defaultdict(list))  # (cfg, kernel) -> counter -> values per dispatch
    for f in sorted(glob.glob(os.path.join(d, "sq_*_*", "pmc_counter_collection.csv"))):
        cfg = os.path.basename(os.path.dirname(f)).split("_")[1]
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], short(r["Kernel_Name"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        for (_, k), cs in per.items():
            for c, v in cs.items():
                acc[(cfg, k)][c].append(v)
    return acc


def main():
    for d in sys.argv[1:]:
        acc = load(d)
        for (cfg, k), cs in sorted(acc.items()):
            m = {c: sum(v) / len(v) for c, v in cs.items()}
            w = m.get("SQ_WAVES") or 0
            out = ["%-4s %-34s" % (cfg, k)]
            if w:
                for c in sorted(m):
                    if c.startswith("SQ_INSTS") or c.startswith("SQ_INST_"):
                        out.append("%s/wave=%.1f" % (c.replace("SQ_INSTS_", "").replace("SQ_", ""), m[c] / w))
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if c in m:
                        out.append("%s=%.0f%%" % (c.replace("SQ_", ""), 100 * m[c] / wc))
                if w:
                    out.append("cyc/wave=%.0f" % (4 * wc / w))
            for c in sorted(m):
                if not (c.startswith("SQ_INSTS") or c.startswith("SQ_INST_") or c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                                                                                 "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
                    out.append("%s=%.4g" % (c, m[c] / w if w and c.startswith("SQ_") else m[c]))
            print(" ".join(out))


if __name__ == "__main__":
    main()
