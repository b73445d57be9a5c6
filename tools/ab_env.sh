#!/bin/bash
# A/B of one environment knob per bench config (grouped batches, no PMC / parity / CPU legs):
#   tools/ab_env.sh TAG "C2 C3" GPC_GROUP_XCD "1 2 3"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:?tag}; CFGS=${2:?configs}; VAR=${3:?variable}; VALUES=${4:?values}
O=gpurun_out/$TAG; mkdir -p "$O"
for c in $CFGS; do for v in $VALUES; do
  env "$VAR=$v" timeout -k 10 300 python -u bench.py --config $c --no-traffic --no-parity --no-cpu-baseline \
    > "$O/b_${c}_$v.json" 2> "$O/b_${c}_$v.err" || { tail -5 "$O/b_${c}_$v.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'config': sys.argv[2], sys.argv[3]: sys.argv[4], 'mpps': d['value'], 'ms_per_step': d['ms_per_step']}))" \
    "$O/b_${c}_$v.json" "$c" "$VAR" "$v" | tee -a "$O/ab.jsonl"
done; done
