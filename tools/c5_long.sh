#!/bin/bash
# Long C5 lines (address churn at 10 000 ops/s with background compaction) next to C3 on one box:
#   tools/c5_long.sh TAG STEPS [GPC_LIB=...]...
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; STEPS=${2:-3000}; shift 2
mkdir -p "$O"
timeout -k 10 300 python -u bench.py --config C3 --no-traffic --no-cpu-baseline > "$O/C3.json" 2> "$O/C3.err" || { tail -5 "$O/C3.err"; exit 1; }
k=0
for set in "" "$@"; do
  k=$((k+1))
  env $set timeout -k 10 600 python -u bench.py --config C5 --steps "$STEPS" --warmup 20 $C5ARGS > "$O/C5_$k.json" 2> "$O/C5_$k.err" \
    || { tail -5 "$O/C5_$k.err"; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
for f in [O + "/C3.json"] + sorted(glob.glob(O + "/C5_*.json")):
    d = json.load(open(f))
    u = d.get("update") or {}
    print(f.split("/")[-1], d["value"], d["ms_per_step"], "elapsed_s=%.1f" % (d["ms_per_step"] * d["steps"] / 1e3),
          {k: u.get(k) for k in ("ops", "ops_per_s", "commits", "op_latency_ms", "commit_ms", "full_builds", "delta_builds",
                                 "background_builds", "overlay_rules_end")})
PY
