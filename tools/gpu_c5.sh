#!/bin/bash
# C5 churn benches (one GPU call): long run at 10k ops/s (spans background compactions) and 1k ops/s.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests (delta/service)" && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread -k "delta or service" > gpurun_out/gpu_tests_c5.log 2>&1 || { tail -20 gpurun_out/gpu_tests_c5.log; exit 1; }
tail -3 gpurun_out/gpu_tests_c5.log
for r in ${CHURN_RATES:-10000 1000}; do
  step "bench C5 rate $r" && timeout -k 10 600 python bench.py --config C5 --churn-rate $r --steps ${C5_STEPS:-400} \
    > gpurun_out/bench_c5_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_c5_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['update'])"
done
echo "== done"
