#!/bin/bash
# Bench lines of C1, C2, C4 (current tree), one JSON line each under gpurun_out/v16/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/v16
for c in C1 C2 C4; do
  echo "== $c ($(date +%T))"
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-traffic \
    > gpurun_out/v16/$c.log 2>&1 || { tail -5 gpurun_out/v16/$c.log; exit 1; }
  tail -1 gpurun_out/v16/$c.log | cut -c1-200
done
