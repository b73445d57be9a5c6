#!/bin/bash
# A/B timing of two library builds ($A, $B under antrea_amd/_build), alternating, configs $CONFIGS.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for rep in 1 2; do
  for v in $A $B; do
    for c in ${CONFIGS:-C3}; do
      GPC_LIB=antrea_amd/_build/$v timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline \
        --no-traffic > gpurun_out/exp/ab_${v}_$c.log 2>&1 || { echo "FAILED $v $c"; tail -5 gpurun_out/exp/ab_${v}_$c.log; exit 1; }
      tail -1 gpurun_out/exp/ab_${v}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['config']['workload'], d['value'], d['kernel_ms'])"
    done
  done
done
echo "== done"
