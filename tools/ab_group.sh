#!/bin/bash
# A/B of the packet grouping pre-pass per bench config: tools/ab_group.sh TAG "C1 C2 C4"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:?tag}; CFGS=${2:-"C1 C2 C3 C4"}
O=gpurun_out/$TAG; mkdir -p "$O"
for c in $CFGS; do for g in -1 1; do
  timeout -k 10 300 python -u bench.py --config $c --group $g --no-traffic --no-parity --no-cpu-baseline \
    > "$O/b_${c}_g$g.json" 2> "$O/b_${c}_g$g.err" || { tail -5 "$O/b_${c}_g$g.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/b_${c}_g$g.json" "$c group=$g"
done; done
