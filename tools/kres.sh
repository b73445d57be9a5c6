#!/bin/bash
# Per-kernel resources of classify.hip (compile-time report, CPU only): VGPRs, spills, scratch
# bytes per lane, LDS bytes, occupancy. Extra hipcc flags (e.g. -DGPC_WAVES_PER_EU=5) pass through.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -I$ROOT/antrea_amd/csrc \
  "$@" -c $ROOT/antrea_amd/csrc/classify.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
rows, cur = [], None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        name = m.group(1)
        t = re.search(r"classify_kernelIL([bi]\d)EL(b\d)ELi(\d)EL(b\d)E", name)
        cur = {"kernel": "classify<mode=%s,svc=%s,stage=%s,sort=%s>" % (t.group(1)[1], t.group(2)[1], t.group(3),
               t.group(4)[1]) if t else re.sub(r"^_ZN3gpc\d+", "", name)[:40]}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"\sVGPRs: (\d+)"), ("vgpr_spill", r"VGPRs Spill: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, l)
        if m and cur is not None:
            cur[key] = int(m.group(1))
print("%-48s %5s %6s %8s %6s %4s" % ("kernel", "VGPR", "spill", "scratch", "LDS", "occ"))
for r in rows:
    print("%-48s %5s %6s %8s %6s %4s" % (r["kernel"], r.get("vgpr"), r.get("vgpr_spill"), r.get("scratch"), r.get("lds"), r.get("occ")))
'
