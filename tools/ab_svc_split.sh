#!/bin/bash
# Service launch split A/B (GPC_SVC_SPLIT=0 / 1) on one box, after the Service GPU tests.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py "tests/test_gpu_fullscale.py::test_device_vs_oracle_fullscale" -m gpu -x -v -k "service or svc or C4 or lb" --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for sp in 1 0; do
  GPC_SVC_SPLIT=$sp timeout -k 10 600 python -u bench.py --config C4 --no-cpu-baseline --no-traffic > "$O/C4_split$sp.json" 2> "$O/C4_split$sp.err" || { tail -5 "$O/C4_split$sp.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/C4_split$sp.json')); print('split $sp', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], (d.get('parity') or {}).get('mismatches'))"
done
