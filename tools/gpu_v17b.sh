#!/bin/bash
# Second v17 session: C3 IPv6, C5 churn @10k ops/s, and an SQ PMC pass on the classify kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/v17
mkdir -p $O
step() { echo "== $1 ($(date +%T))"; }
step c3v6 && timeout -k 10 400 python bench.py --config C3 --family 6 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic \
  > $O/c3v6.log 2>&1 || { tail -5 $O/c3v6.log; exit 1; }
tail -1 $O/c3v6.log | cut -c1-200
step "c5 10000" && timeout -k 10 600 python bench.py --config C5 --churn-rate 10000 --steps 400 \
  > $O/c5_10000.log 2>&1 || { tail -5 $O/c5_10000.log; exit 1; }
tail -1 $O/c5_10000.log | cut -c1-200
step "rocprof SQ" && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES --kernel-include-regex classify \
  -d $O/prof_sq -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --no-traffic > $O/prof_sq.log 2>&1 || { tail -5 $O/prof_sq.log; exit 1; }
find $O/prof_sq -name "*.csv"
echo "== done"
