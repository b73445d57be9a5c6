#!/bin/bash
# Counter-aggregation experiment: GPU counter tests, then C2 / C3 bench with wave-aggregated
# counters (default build), per-lane atomics (libgpc_noagg.so) and counters off.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k counters \
  > gpurun_out/exp/tests.log 2>&1 || { tail -30 gpurun_out/exp/tests.log; exit 1; }
tail -3 gpurun_out/exp/tests.log
B=antrea_amd/_build
run() {  # name, config, extra, env...
  local name=$1 cfg=$2 extra=$3; shift 3
  echo "== $name ($(date +%T))"
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-traffic $extra \
    > gpurun_out/exp/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/exp/$name.log; exit 1; }
  tail -1 gpurun_out/exp/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])"
}
run c2_agg C2 "" GPC_LIB=$B/libgpc.so
run c2_noagg C2 "" GPC_LIB=$B/libgpc_noagg.so
run c2_nocount C2 --no-count GPC_LIB=$B/libgpc.so
run c3_agg C3 "" GPC_LIB=$B/libgpc.so
run c3_noagg C3 "" GPC_LIB=$B/libgpc_noagg.so
run c3_nocount C3 --no-count GPC_LIB=$B/libgpc.so
echo "== done"
