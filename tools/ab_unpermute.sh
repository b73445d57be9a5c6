#!/bin/bash
# Un-permute A/B (GPC_GROUP_UNPERMUTE): grouping parity tests, then per-kernel times and bench lines
# of C3 and C2 with the ingress verdicts scattered by the ingress launch (0) or un-permuted (1).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:-up}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_group.py} -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/kt_env.sh ${TAG}_kt3 C3 "GPC_GROUP_UNPERMUTE=0 GPC_GROUP_UNPERMUTE=1" || exit 1
bash tools/kt_env.sh ${TAG}_kt2 C2 "GPC_GROUP_UNPERMUTE=0 GPC_GROUP_UNPERMUTE=1" || exit 1
bash tools/sweep_env.sh ${TAG}_b3 C3 "GPC_GROUP_UNPERMUTE=1 GPC_GROUP_UNPERMUTE=0 GPC_GROUP_UNPERMUTE=1" || exit 1
