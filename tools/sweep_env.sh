#!/bin/bash
# Bench one config under several environment settings: tools/sweep_env.sh TAG CONFIG "A=1,B=2 A=0" [bench args]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:?tag}; CFG=${2:-C3}; SETS=$3; shift 3
O=gpurun_out/$TAG; mkdir -p "$O"
k=0
for set in $SETS; do
  k=$((k+1))
  env $(echo "$set" | tr ',' ' ') timeout -k 10 300 python -u bench.py --config $CFG --no-traffic --no-parity --no-cpu-baseline "$@" \
    > "$O/b_${CFG}_$k.json" 2> "$O/b_${CFG}_$k.err" || { tail -5 "$O/b_${CFG}_$k.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/b_${CFG}_$k.json" "$CFG $set"
done
