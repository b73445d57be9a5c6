#!/bin/bash
# Quick bench lines of several configs on one box (no PMC passes / CPU baseline):
#   tools/ab_quick.sh TAG CFG... (v6 = C3 in IPv6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; shift; mkdir -p "$O"
for c in "$@"; do
  if [ "$c" = v6 ]; then a="--family 6"; else a="--config $c"; fi
  timeout -k 10 600 python -u bench.py $a --no-cpu-baseline --no-traffic > "$O/$c.json" 2> "$O/$c.err" || { tail -5 "$O/$c.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], (d.get('parity') or {}).get('mismatches'))"
done
