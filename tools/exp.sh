#!/bin/bash
# Kernel experiment sweep (one GPU call): bench variants, one JSON line each.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
run() {  # name, env...
  local name=$1; shift
  echo "== $name ($(date +%T))"
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic $EXTRA \
    > gpurun_out/exp/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/exp/$name.log; exit 1; }
  tail -1 gpurun_out/exp/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['roofline']['lines_per_packet'])"
}
B=antrea_amd/_build
for v in ${VARIANTS:-w4}; do
  if [ "$v" = base ]; then run base GPC_LIB=$B/libgpc.so; else run $v GPC_LIB=$B/libgpc_$v.so; fi
done
echo "== done"
