#!/bin/bash
# PC sampling (beta) of the classify kernel on a reduced packet count.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 100 --kernel-trace -d gpurun_out/pcs -o pcs --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --packets 16777216 > gpurun_out/pcs.log 2>&1
rc=$?
tail -5 gpurun_out/pcs.log
ls -la gpurun_out/pcs/ 2>/dev/null | head
exit $rc
