cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_fullscale.py tests/test_gpu_e2e.py -k "c2g or C1 or e2e" -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_env.sh r05h C1 "X=bitset GPC_NO_BITSET=1" --steps 20 || exit 1
bash tools/ab_quick.sh r05h C3 C4 C2 || exit 1
timeout -k 10 600 python -u bench.py --config C2g --no-parity --no-cpu-baseline --no-traffic > $O/C2g.json 2> $O/C2g.err || { tail -5 $O/C2g.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/C2g.json')); print('C2g', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['config']['image_mb'], d['config']['build_s'])"
