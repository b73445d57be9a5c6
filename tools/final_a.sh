#!/bin/bash
# Round-end evidence, part A: the default bench line (C3, PMC passes, parity, CPU baseline) with its
# counter CSVs kept, then a kernel-trace profile of the same workload.  tools/final_a.sh TAG
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; mkdir -p "$O"
timeout -k 10 900 python -u bench.py --keep-pmc "$O/pmc" > "$O/c3_bench.json" 2> "$O/c3_bench.err" || { tail -5 "$O/c3_bench.err"; exit 1; }
cat "$O/c3_bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 \
  --no-traffic --no-cpu-baseline --no-parity > "$O/kt.log" 2>&1 || { tail -5 "$O/kt.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$O/c3_kernel_stats.csv"
head -8 "$O/c3_kernel_stats.csv"
