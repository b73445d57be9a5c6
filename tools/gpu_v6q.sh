#!/bin/bash
# IPv6 GPU parity tests + the C3 IPv6 bench line (quick loop for the LPM work).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
timeout -k 10 400 python -u -m pytest tests -m gpu -k "ipv6 or smoke" -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/exp/t6.log 2>&1 || { tail -30 gpurun_out/exp/t6.log; exit 1; }
tail -1 gpurun_out/exp/t6.log
timeout -k 10 400 python bench.py --config C3 --family 6 --steps 5 --warmup 2 --no-cpu-baseline --no-traffic \
  > gpurun_out/exp/c3v6.log 2>&1 || { tail -5 gpurun_out/exp/c3v6.log; exit 1; }
tail -1 gpurun_out/exp/c3v6.log
