#!/bin/bash
# Kernel-trace stats of one bench config for this tree and the worktree _wt_old (A/B of a change).
#   tools/kt_cmp.sh TAG CONFIG [bench args]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}; CFG=$2; shift 2
O=$PWD/gpurun_out/$TAG; mkdir -p "$O"
for t in new old; do
  d=.; extra=("$@"); [ $t = old ] && { d=_wt_old; extra=(); }  # extra bench args: this tree only
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_$t" -o kt --output-format csv -- \
    python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-parity "${extra[@]}" > "$O/kt_$t.log" 2>&1) || exit 1
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'gpc' in r['Name']: print(sys.argv[2], r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,3))
" "$O/kt_$t/kt_kernel_stats.csv" $t
done
