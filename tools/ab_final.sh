#!/bin/bash
# C5 with the delta-epoch grouping rule, then ungrouped C3 under composite sizings (extra bits 0/1/2).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p "$O"
one() {  # name, env..., then bench args after --
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-traffic "$@" > "$O/$name.json" 2> "$O/$name.err" || { tail -5 "$O/$name.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], (d.get('parity') or {}).get('mismatches'), d['config'].get('image_mb'), d['config']['packet_grouping'])"
}
one C5 X=1 -- --config C5
for x in 0 1 2; do one C3_x$x GPC_COMPOSITE_EXTRA_BITS=$x -- --config C3 --no-parity; done
