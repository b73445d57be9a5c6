#!/bin/bash
# Un-permute A/B (GPC_GROUP_UNPERMUTE): grouping / full-scale / concurrency GPU tests, then per-kernel
# times of C3 and bench lines of C3 and C5 with the ingress verdicts stored at the caller index by the
# ingress launch (0) or joined and put in caller order by the un-permute launch (1).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:-up}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_group.py} -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/kt_env.sh ${TAG}_kt3 C3 "GPC_GROUP_UNPERMUTE=0 GPC_GROUP_UNPERMUTE=1" || exit 1
bash tools/sweep_env.sh ${TAG}_b3 C3 "GPC_GROUP_UNPERMUTE=1 GPC_GROUP_UNPERMUTE=0" || exit 1
bash tools/sweep_env.sh ${TAG}_b5 C5 "GPC_GROUP_UNPERMUTE=1 GPC_GROUP_UNPERMUTE=0" || exit 1
for f in gpurun_out/${TAG}_b5/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['update']['op_latency_ms'], d['update']['commit_ms'])" $f; done
