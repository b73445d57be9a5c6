#!/bin/bash
# One GPU session: parity tests, smoke, bench (with CPU baseline), rocprofv3 kernel trace + PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
step bench && timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
step "rocprof kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic \
  > gpurun_out/prof_kt.log 2>&1 || exit $?
tail -1 gpurun_out/prof_kt.log
step "rocprof SQ" && timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES --kernel-include-regex classify \
  -d gpurun_out/prof_sq -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --no-traffic > gpurun_out/prof_sq.log 2>&1 || exit $?
step "rocprof TCC" && timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex classify \
  -d gpurun_out/prof_tcc -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --no-traffic > gpurun_out/prof_tcc.log 2>&1 || exit $?
find gpurun_out -name "*.csv" | head -20
echo "== done"
