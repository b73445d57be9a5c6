cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_ipv6_delta.py -k "ipv6" -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for set in X=default GPC_V6_LEAF_LENS=8 GPC_V6_LEAF_LENS=2; do
  env $set timeout -k 10 600 python -u bench.py --family 6 --no-cpu-baseline --no-traffic --no-parity > $O/v6_$set.json 2> $O/v6_$set.err || { tail -5 $O/v6_$set.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'], d['config']['image_mb'], d['config']['build_s'])" $O/v6_$set.json $set
done
timeout -k 10 900 python -u bench.py --family 6 --keep-pmc $O/pmc_v6 > $O/v6.json 2> $O/v6.err || { tail -5 $O/v6.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('v6', d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['roofline']['kernels'].get('v6_codes'))" $O/v6.json
timeout -k 10 600 python -u bench.py --family 6 --v6-embed multi48 --no-cpu-baseline --no-traffic > $O/v6m48.json 2> $O/v6m48.err || { tail -5 $O/v6m48.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('multi48', d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'])" $O/v6m48.json
