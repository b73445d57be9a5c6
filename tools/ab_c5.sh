#!/bin/bash
# C5 (churn, delta epochs) A/B of two library builds on one box: the product libgpc.so and
# GPC_LIB=antrea_amd/_build/libgpc_$2.so, after the churn device-vs-oracle test.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${1:?tag}; V=${2:?variant}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest "tests/test_gpu_fullscale.py::test_device_vs_oracle_after_churn_c3" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for lib in product $V product $V; do
  if [ $lib = product ]; then unset GPC_LIB; else export GPC_LIB=$PWD/antrea_amd/_build/libgpc_$V.so; fi
  timeout -k 10 600 python -u bench.py --config C5 --no-cpu-baseline --no-traffic > "$O/C5_$lib.json" 2> "$O/C5_$lib.err" || { tail -5 "$O/C5_$lib.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/C5_$lib.json')); print('$lib', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['update']['overlay_rules_end'])"
done
