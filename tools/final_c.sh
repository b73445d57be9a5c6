#!/bin/bash
# Round-end evidence, part C: the churn lines after the last kernel changes -- C4 (Service stage),
# C5 with the mixed op stream (parity stamp) and with the uniform one.  tools/final_c.sh TAG [C5_STEPS]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; mkdir -p "$O"
echo "== C4 $(date +%T)"
timeout -k 10 400 python -u bench.py --config C4 > "$O/C4_bench.json" 2> "$O/C4_bench.err" || { tail -5 "$O/C4_bench.err"; exit 1; }
echo "== C5 mixed $(date +%T)"
timeout -k 10 700 python -u bench.py --config C5 --steps "${2:-3000}" --warmup 20 > "$O/C5_bench.json" 2> "$O/C5_bench.err" || { tail -5 "$O/C5_bench.err"; exit 1; }
echo "== C5 uniform $(date +%T)"
timeout -k 10 700 python -u bench.py --config C5 --churn-mix uniform --steps "${2:-3000}" --warmup 20 > "$O/C5u_bench.json" 2> "$O/C5u_bench.err" || { tail -5 "$O/C5u_bench.err"; exit 1; }
for f in C4 C5 C5u; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('kernel_ms_by_launch'), (d.get('parity') or {}).get('mismatches'))" "$O/${f}_bench.json" "$f"
done
