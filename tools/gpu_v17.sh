#!/bin/bash
# Round-1 closing GPU session for the current tree: parity tests, smoke, default bench (CPU baseline +
# PMC traffic), rocprofv3 kernel-trace stats, then C1/C2/C4 bench lines. Output under gpurun_out/v17/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/v17
mkdir -p $O
step() { echo "== $1 ($(date +%T))"; }
step "gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench && timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
step "rocprof kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic \
  > $O/prof_kt.log 2>&1 || { tail -5 $O/prof_kt.log; exit 1; }
for c in C1 C2 C4; do
  step $c
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-traffic \
    > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
  tail -1 $O/$c.log | cut -c1-200
done
find $O -name "*stats*.csv"
echo "== done"
