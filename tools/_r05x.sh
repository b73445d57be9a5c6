cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
run() {  # tag, lib ('' = product), bench args
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export GPC_LIB=antrea_amd/_build/libgpc_$lib.so; else unset GPC_LIB; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic --no-parity --steps 20 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'])" $O/$tag.json $tag
}
run C3_u4 "" --config C3
run C3_nocount "" --config C3 --no-count
run C3_u2 u2 --config C3
run C3_u3 u3 --config C3
run C3_u6 u6 --config C3
run C2_u4 "" --config C2
run C2_u6 u6 --config C2
run C1_u4 "" --config C1
run C1_u3 u3 --config C1
run C1_u6 u6 --config C1
