#!/bin/bash
# Round-end evidence, part B: the other configs' bench lines (C1, C2, C2g, C4, C3 in IPv6; PMC passes,
# parity, CPU baseline) and a long C5 line.  tools/final_b.sh TAG [C5_STEPS]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; mkdir -p "$O"
for c in C1 C2 C2g C4 v6; do
  if [ "$c" = v6 ]; then a="--family 6"; else a="--config $c"; fi
  echo "== $c $(date +%T)"
  timeout -k 10 400 python -u bench.py $a > "$O/${c}_bench.json" 2> "$O/${c}_bench.err" || { tail -5 "$O/${c}_bench.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('parity'), (d.get('cpu_baseline') or {}).get('value'), d['roofline'].get('frac'))" "$O/${c}_bench.json" "$c"
done
echo "== C5 $(date +%T)"
timeout -k 10 600 python -u bench.py --config C5 --steps "${2:-2000}" --warmup 20 > "$O/C5_bench.json" 2> "$O/C5_bench.err" || { tail -5 "$O/C5_bench.err"; exit 1; }
cat "$O/C5_bench.json"
