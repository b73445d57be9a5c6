#!/bin/bash
# GPU parity tests, then short bench lines for the configs in $CONFIGS (default C2 C3).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/exp/tests.log 2>&1 || { tail -30 gpurun_out/exp/tests.log; exit 1; }
  tail -1 gpurun_out/exp/tests.log
fi
for c in ${CONFIGS:-C2 C3}; do
  echo "== $c ($(date +%T))"
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-traffic $EXTRA \
    > gpurun_out/exp/$c.log 2>&1 || { echo "FAILED $c"; tail -5 gpurun_out/exp/$c.log; exit 1; }
  tail -1 gpurun_out/exp/$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['kernel_ms'], d['config']['image_mb'])"
done
echo "== done"
