cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ze; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for c in C3 C2 C4; do
timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline --no-traffic --steps 20 > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['config']['image_mb'])" $O/$c.json $c
done
