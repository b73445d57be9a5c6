#!/bin/bash
# A/B runner for the gpurun box (from the repo root): one bench.py run per variant, in order.
#   tools/ab.sh TAG 'label|ENV=V ENV2=V|bench.py args' ...
# e.g. tools/ab.sh r06b 'base||' 'split|GPC_SPLIT_STORE=1|' 'v6|GPC_SPLIT_STORE=1|--family 6 --no-traffic'
# Every variant runs `bench.py --no-cpu-baseline --keep-pmc gpurun_out/TAG/pmc_LABEL <args>` under its
# own time limit (AB_TIMEOUT, default 400 s); the line goes to gpurun_out/TAG/LABEL.json and a one-line
# summary (ms/step, launches, parity mismatches, dominant-kernel frac, fabric bytes per packet) is
# printed. The first failing variant ends the session (no retries).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
for v in "$@"; do
  IFS='|' read -r label envs args <<< "$v"
  echo "== $label ($(date +%T)) env: $envs args: $args"
  # shellcheck disable=SC2086
  timeout -k 10 "${AB_TIMEOUT:-400}" env $envs python3 -u bench.py --no-cpu-baseline --keep-pmc "$O/pmc_$label" $args \
    > "$O/$label.json" 2> "$O/$label.err" || { echo "variant $label failed"; tail -20 "$O/$label.err"; exit 1; }
  python3 - "$O/$label.json" "$label" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
ks = {k: (v.get("ms"), v.get("bytes_per_packet")) for k, v in (r.get("kernels") or {}).items()}
print(sys.argv[2], "ms/step", d["ms_per_step"], "Mpps", d["value"], "parity", (d.get("parity") or {}).get("mismatches"),
      "frac", r.get("frac"), "B/pkt", (r.get("step") or {}).get("traffic_per_packet"), ks, flush=True)
PY
done
