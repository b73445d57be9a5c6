#!/bin/bash
# GPU tests + C3 / C4 bench + C5 churn bench (one GPU call). Every GPU step has its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -18 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
step "bench C3" && timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
step "bench C4" && timeout -k 10 600 python bench.py --config C4 --no-traffic > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log
for r in ${CHURN_RATES:-10000}; do
  step "bench C5 rate $r" && timeout -k 10 600 python bench.py --config C5 --churn-rate $r --steps 100 \
    > gpurun_out/bench_c5_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_c5_$r.log
done
echo "== done"
