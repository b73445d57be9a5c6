#!/bin/bash
# Composite driver sizing A/B on one box: GPC_COMPOSITE_EXTRA_BITS 1 / 2 on C3 and C2, then C1 and C4
# with and without the composite index.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; mkdir -p "$O"
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-traffic --no-parity $BARGS > "$O/$name.json" 2> "$O/$name.err" || exit 1
}
for cfg in C3 C2; do
  BARGS="--config $cfg"
  run ${cfg}_x1 GPC_COMPOSITE=1 GPC_COMPOSITE_EXTRA_BITS=1
  run ${cfg}_x2 GPC_COMPOSITE=1 GPC_COMPOSITE_EXTRA_BITS=2
done
for cfg in C1 C4; do
  BARGS="--config $cfg"
  run ${cfg}_x1 GPC_COMPOSITE=1 GPC_COMPOSITE_EXTRA_BITS=1
  run ${cfg}_plain GPC_COMPOSITE=0
done
for f in "$O"/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config'].get('image_mb'), d['kernel_ms_by_launch'])"; done
