#!/bin/bash
# A/B of the packet grouping pre-pass per bench config:
#   tools/ab_group.sh TAG "C1 C2 C4" ["plain addr scan"]
# plain = ungrouped, addr = grouped by nw_src top bits, scan = grouped by scan lengths (GPC_GROUP_KEY).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:?tag}; CFGS=${2:-"C1 C2 C3 C4"}; VARIANTS=${3:-"plain addr scan"}
O=gpurun_out/$TAG; mkdir -p "$O"
for c in $CFGS; do for v in $VARIANTS; do
  case $v in plain) g=-1; k=0 ;; addr) g=1; k=1 ;; scan) g=1; k=2 ;; *) echo "bad variant $v"; exit 2 ;; esac
  GPC_GROUP_KEY=$k timeout -k 10 300 python -u bench.py --config $c --group $g --no-traffic --no-parity --no-cpu-baseline \
    > "$O/b_${c}_$v.json" 2> "$O/b_${c}_$v.err" || { tail -5 "$O/b_${c}_$v.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/b_${c}_$v.json" "$c $v"
done; done
