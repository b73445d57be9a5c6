#!/bin/bash
# A/B of the composite driver index (GPC_COMPOSITE=0 / 1) on one box: C3 and C2 lines.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p "$O"
for cfg in C3 C2; do
  GPC_COMPOSITE=1 timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline --no-traffic > "$O/${cfg}_composite.json" 2> "$O/${cfg}_composite.err" || exit 1
  GPC_COMPOSITE=1 GPC_COMPOSITE_EXTRA_BITS=1 timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline --no-traffic --no-parity > "$O/${cfg}_composite_x1.json" 2> "$O/${cfg}_composite_x1.err" || exit 1
  GPC_COMPOSITE=0 timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline --no-traffic --no-parity > "$O/${cfg}_plain.json" 2> "$O/${cfg}_plain.err" || exit 1
done
for f in "$O"/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d.get('parity'))"; done
