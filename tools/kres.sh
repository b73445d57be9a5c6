#!/bin/bash
# Per-kernel VGPRs / spills / occupancy of classify.hip (compile-time resource report, CPU only).
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include -I/root/repo/antrea_amd/csrc \
  "$@" -c /root/repo/antrea_amd/csrc/classify.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re,sys
cur=None
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: cur=m.group(1); print(); print(re.sub(r"EEEvNS.*","",cur.replace("_ZN3gpc15classify_kernelI","")),end=" ")
    for k in ("VGPRs","VGPRs Spill","SGPRs Spill","Occupancy \\[waves/SIMD\\]"):
        m=re.search(r"\s"+k+r": (\d+)",l)
        if m: print(k.split()[0]+("S" if "Spill" in k else "")+"="+m.group(1),end=" ")
print()'
