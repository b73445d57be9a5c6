#!/bin/bash
# One GPU session on the gpurun box (run from the repo root):
#   tools/gpu_session.sh TAG [STEPS...]
# STEPS (default "tests smoke bench kt"):
#   build   python -m antrea_amd.build --force on the box (every object recompiled from source there;
#           the later steps then load the box-built library)
#   tests   pytest -m gpu (one process, per-test timeout)
#   smoke   __graft_entry__.smoke()
#   bench   python bench.py (default C3 line: PMC passes, parity stamp, CPU baseline)
#   cfg:X   bench.py --config X (C1, C2, C2g, C4, C5) ; v6 = C3 in IPv6, v6m48 = the same over four /48s
#   kt      rocprofv3 --kernel-trace --stats over a short bench run
#   sq[:X]  rocprofv3 SQ counters (config X, default C3) ; tcc[:X] TCC hit / miss / EA read requests
#   fetch / write  FETCH_SIZE / WRITE_SIZE of C3
# Outputs under gpurun_out/TAG/. Every GPU step has its own time limit; the script stops at the
# first failure (no retries).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}
shift
STEPS=${*:-tests smoke bench kt}
O=gpurun_out/$TAG
mkdir -p "$O"
step() { echo "== $1 ($(date +%T))"; }
KT_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-parity"
pmc() {  # name, config, counters...
  local name=$1 cfg=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "classify|unpermute" -d "$O/pmc_${name}_$cfg" -o pmc \
    --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-parity \
    --config $cfg > "$O/pmc_${name}_$cfg.log" 2>&1
}
for s in $STEPS; do
  case $s in
    build)
      step build
      timeout -k 10 900 python -u -m antrea_amd.build --force > "$O/build.log" 2>&1 || { tail -20 "$O/build.log"; exit 1; }
      tail -1 "$O/build.log"; sha256sum antrea_amd/_build/libgpc.so >> "$O/build.log" ;;
    tests)
      step tests
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --durations=30 --timeout 400 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1; rc=$?
      tail -5 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      step smoke
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
      tail -1 "$O/smoke.log" ;;
    bench)
      step bench
      timeout -k 10 900 python -u bench.py --keep-pmc "$O/pmc_bench" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
      cat "$O/bench.json" ;;
    cfg:*)
      c=${s#cfg:}; step "bench $c"
      case $c in
        v6) a="--family 6" ;;
        v6m48) a="--family 6 --v6-embed multi48 --no-cpu-baseline" ;;
        C2g) a="--config C2g --no-cpu-baseline" ;;
        C5) a="--config C5 --steps ${C5_STEPS:-3500} --warmup 20" ;;
        *) a="--config $c" ;;
      esac
      timeout -k 10 900 python -u bench.py $a --keep-pmc "$O/pmc_$c" > "$O/bench_$c.json" 2> "$O/bench_$c.err" || { tail -20 "$O/bench_$c.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], (d.get('parity') or {}).get('mismatches'))" "$O/bench_$c.json" $c ;;
    kt)
      step "rocprof kernel trace"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- \
        python3 bench.py $KT_ARGS > "$O/kt.log" 2>&1 || exit $?
      tail -1 "$O/kt.log" ;;
    sq|sq:*)
      c=${s#sq}; c=${c#:}; c=${c:-C3}; step "rocprof SQ $c"
      pmc sq $c SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_INSTS_VMEM_RD SQ_WAVES || exit $? ;;
    tcc|tcc:*)
      c=${s#tcc}; c=${c#:}; c=${c:-C3}; step "rocprof TCC $c"
      pmc tcc $c TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum || exit $? ;;
    fetch)
      step "rocprof FETCH_SIZE"; pmc fetch C3 FETCH_SIZE || exit $? ;;
    write)
      step "rocprof WRITE_SIZE"; pmc write C3 WRITE_SIZE || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
find "$O" -name "*.csv" | head -40
echo "== done"
