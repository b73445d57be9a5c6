#!/bin/bash
# C3 IPv4 bench (with PMC traffic) and C3 IPv6 bench of the current tree.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/v15
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/v15/c3.log 2>&1 || { tail -5 gpurun_out/v15/c3.log; exit 1; }
tail -1 gpurun_out/v15/c3.log
timeout -k 10 400 python bench.py --config C3 --family 6 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic \
  > gpurun_out/v15/c3v6.log 2>&1 || { tail -5 gpurun_out/v15/c3v6.log; exit 1; }
tail -1 gpurun_out/v15/c3v6.log
