#!/bin/bash
# Sweep of the packet grouping knobs (GPC_GROUP_TILE / GPC_GROUP_SHIFT) on one bench config.
#   tools/sweep_group.sh TAG CONFIG "tile:shift tile:shift ..."
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:?tag}; CFG=${2:-C3}; SETS=${3:-"16384:24"}
O=gpurun_out/$TAG; mkdir -p "$O"
for ts in $SETS; do
  t=${ts%:*}; s=${ts#*:}
  GPC_GROUP_TILE=$t GPC_GROUP_SHIFT=$s timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --no-traffic --no-parity \
    --no-cpu-baseline > "$O/b_${CFG}_$t_$s.json" 2> "$O/b_${CFG}_$t_$s.err" || { tail -5 "$O/b_${CFG}_$t_$s.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/b_${CFG}_$t_$s.json" "$CFG tile=$t shift=$s"
done
