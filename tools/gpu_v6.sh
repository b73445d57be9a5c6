#!/bin/bash
# GPU parity tests, then C3 IPv4 and C2 / C3 IPv6 bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/exp/tests.log 2>&1 || { tail -40 gpurun_out/exp/tests.log; exit 1; }
tail -3 gpurun_out/exp/tests.log
run() {  # name, args
  local name=$1; shift
  echo "== $name ($(date +%T))"
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic "$@" > gpurun_out/exp/$name.log 2>&1 \
    || { echo "FAILED $name"; tail -5 gpurun_out/exp/$name.log; exit 1; }
  tail -1 gpurun_out/exp/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['config'].get('family', 4), d['value'], d['kernel_ms'], d['config']['image_mb'], d['roofline']['lines_per_packet'])"
}
run c3 --config C3
run c3v6 --config C3 --family 6
run c2v6 --config C2 --family 6
echo "== done"
