"""FETCH_SIZE calibration for gather access patterns (run on the GPU box from the repo root).

    python3 tools/fetch_calib.py [--out profiles/r05_fetch_calib]

Runs tools/_build/fetch_calib (tools/fetch_calib.hip, built here with hipcc by --build) plainly for
its timings, then under two rocprofv3 PMC passes (FETCH_SIZE; TCC_EA0_RDREQ_sum + TCC_EA0_RDREQ_32B_sum
+ TCC_HIT_sum + TCC_MISS_sum), for a 128 MiB buffer (Infinity-Cache resident, like the C3 image) and
a 1 GiB one (HBM). Every kernel runs twice (the first fills the caches); the table uses the second
dispatch. Output: per kernel the known distinct bytes, FETCH_SIZE bytes, their ratio (the factor
FETCH_SIZE must be multiplied by to give the bytes moved), and the EA read requests per distinct
128-B line.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "_build", "fetch_calib")


def build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    os.path.join(ROOT, "tools", "fetch_calib.hip"), "-o", BIN], check=True)


def run_plain(mib):
    out = subprocess.run([BIN, str(mib)], check=True, capture_output=True, text=True, timeout=120).stdout
    rows = {}
    for line in out.splitlines():
        if line.startswith("#"):
            continue
        k, known, ms = line.split("\t")
        rows[k] = {"known_bytes": int(known), "ms": float(ms)}
    return rows


def run_pmc(mib, counters):
    d = tempfile.mkdtemp(prefix="fcal_")
    cmd = ["rocprofv3", "--pmc"] + counters + ["-d", d, "-o", "pmc", "--output-format", "csv", "--", BIN, str(mib)]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=120)
    per = {}  # kernel -> dispatch id -> {counter: value}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
                per.setdefault(k, {}).setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return {k: v[max(v)] for k, v in per.items()}  # the second (warm) dispatch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/fetch_calib")
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build or not os.path.exists(BIN):
        build()
    os.makedirs(a.out, exist_ok=True)
    table = {}
    for mib in (128, 1024):
        rows = run_plain(mib)
        f = run_pmc(mib, ["FETCH_SIZE"])
        t = run_pmc(mib, ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_HIT_sum", "TCC_MISS_sum"])
        for k, r in rows.items():
            fs = f.get(k, {}).get("FETCH_SIZE")
            tc = t.get(k, {})
            lines = r["known_bytes"] / 128.0
            r["fetch_size_bytes"] = fs * 1024.0 if fs is not None else None
            r["known_over_fetch_size"] = round(r["known_bytes"] / r["fetch_size_bytes"], 3) if fs else None
            for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_HIT_sum", "TCC_MISS_sum"):
                if c in tc:
                    r[c] = tc[c]
            if "TCC_EA0_RDREQ_sum" in tc:
                r["rdreq_per_line"] = round(tc["TCC_EA0_RDREQ_sum"] / lines, 3)
            if "TCC_MISS_sum" in tc:
                r["miss_per_line"] = round(tc["TCC_MISS_sum"] / lines, 3)
            r["gbs_known"] = round(r["known_bytes"] / (r["ms"] / 1e3) / 1e9, 1)
        table["%d_MiB" % mib] = rows
    with open(os.path.join(a.out, "fetch_calib.json"), "w") as fh:
        json.dump(table, fh, indent=1)
    for buf, rows in table.items():
        print("buffer", buf)
        print("%-12s %14s %14s %8s %9s %9s %9s" % ("kernel", "known B", "FETCH_SIZE B", "known/FS", "rdreq/ln", "miss/ln",
                                                  "GB/s"))
        for k, r in rows.items():
            print("%-12s %14d %14s %8s %9s %9s %9s" % (k, r["known_bytes"], "%.0f" % r["fetch_size_bytes"] if r["fetch_size_bytes"] else "-",
                                                       r["known_over_fetch_size"], r.get("rdreq_per_line"),
                                                       r.get("miss_per_line"), r["gbs_known"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
