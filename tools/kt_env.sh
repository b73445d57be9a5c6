#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of one bench config under several environment
# settings: tools/kt_env.sh TAG CONFIG "A=1,B=2 A=0" [bench args]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}; CFG=$2; SETS=$3; shift 3
O=$PWD/gpurun_out/$TAG; mkdir -p "$O"
k=0
for set in $SETS; do
  k=$((k+1))
  env $(echo "$set" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_$k" -o kt --output-format csv -- \
    python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-parity "$@" > "$O/kt_$k.log" 2>&1 || exit 1
  python3 -c "
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'gpc' in r['Name']]
print(sys.argv[2], ' | '.join('%s %.3f' % (r['Name'].split('(')[0].replace('void gpc::','')[:40], float(r['AverageNs'])/1e6) for r in rows))
" "$O/kt_$k/kt_kernel_stats.csv" "$set"
done
