cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
for lib in default w5; do
  if [ $lib = default ]; then unset GPC_LIB; else export GPC_LIB=antrea_amd/_build/libgpc_$lib.so; fi
  for c in C3 C1 C2; do
    timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-traffic --no-parity --steps 20 > $O/${c}_$lib.json 2> $O/${c}_$lib.err || { tail -5 $O/${c}_$lib.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'])" $O/${c}_$lib.json "$c $lib"
  done
  timeout -k 10 400 python -u bench.py --config C5 --no-cpu-baseline --no-traffic --steps 1500 --warmup 20 > $O/C5_$lib.json 2> $O/C5_$lib.err || { tail -5 $O/C5_$lib.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['update']['ops_per_s'])" $O/C5_$lib.json "C5 $lib"
done
