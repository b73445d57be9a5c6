#!/bin/bash
# SQ instruction-mix / stall counters per classify launch, several configs, several counter sets:
#   tools/sq_profile.sh TAG "C1 C2 C3" [SET...]
# SET = a comma-separated counter list (one rocprofv3 --pmc pass each; <= 8 SQ counters);
# default: the wave-cycle / wait / instruction-count set. Outputs gpurun_out/TAG/sq_<cfg>_<k>/.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}; CFGS=${2:-C3}; shift 2
SETS=${*:-SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_WAVES}
O=gpurun_out/$TAG; mkdir -p "$O"
for c in $CFGS; do
  if [ "$c" = v6 ]; then a="--family 6"; else a="--config $c"; fi
  k=0
  for s in $SETS; do
    k=$((k+1))
    echo "== $c pass $k: $s ($(date +%T))"
    timeout -s KILL 300 rocprofv3 --pmc $(echo "$s" | tr ',' ' ') --kernel-include-regex "classify|unpermute|group" \
      -d "$O/sq_${c}_$k" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      --no-traffic --no-parity $a > "$O/sq_${c}_$k.log" 2>&1 || { tail -5 "$O/sq_${c}_$k.log"; exit 1; }
  done
done
echo "== done"
