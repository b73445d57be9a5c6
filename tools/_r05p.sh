cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=5 > $O/gpu_tests.log 2>&1; rc=$?
tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for c in C3 C1 C2; do
timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline --no-traffic --steps 20 > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'])" $O/$c.json $c
done
