#!/bin/bash
# GPU tests + one bench line per BASELINE config (C1 plumbing, C2, C3 headline, C4 Services).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
step "bench C1" && timeout -k 10 300 python bench.py --config C1 --packets 1048576 --steps 50 --no-traffic --no-cpu-baseline \
  > gpurun_out/bench_c1.log 2>&1 || exit $?
step "bench C2" && timeout -k 10 600 python bench.py --config C2 --no-traffic --cpu-seconds 10 > gpurun_out/bench_c2.log 2>&1 || exit $?
step "bench C3" && timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
step "bench C4" && timeout -k 10 600 python bench.py --config C4 --no-traffic > gpurun_out/bench_c4.log 2>&1 || exit $?
for f in bench_c1 bench_c2 bench bench_c4; do
  tail -1 gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['kernel_ms'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
done
echo "== done"
