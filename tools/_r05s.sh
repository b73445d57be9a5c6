cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for c in C3 C4 C1; do
timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline --no-traffic --steps 20 > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'])" $O/$c.json $c
done
timeout -k 10 400 python -u bench.py --config C5 --no-cpu-baseline --no-traffic --steps 1500 --warmup 20 > $O/C5.json 2> $O/C5.err || { tail -5 $O/C5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('C5', d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['update']['ops_per_s'])" $O/C5.json
