cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
bash tools/sweep_env.sh r05i C3 "X=default GPC_NO_BITSET=1" --steps 20 || exit 1
timeout -k 10 900 python -u bench.py --config C1 --keep-pmc $O/pmc_c1 > $O/C1.json 2> $O/C1.err || { tail -5 $O/C1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/C1.json')); print('C1', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['roofline']['frac'])"
timeout -k 10 900 python -u bench.py --family 6 --keep-pmc $O/pmc_v6 > $O/v6.json 2> $O/v6.err || { tail -5 $O/v6.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/v6.json')); print('v6', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['roofline']['kernels'].get('v6_codes'))"
GPC_COMPACT_DEBUG=1 timeout -k 10 700 python -u bench.py --config C5 --steps 3500 --warmup 20 > $O/C5.json 2> $O/C5.err || { tail -5 $O/C5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/C5.json')); u=d['update']; print('C5', d['value'], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], u['ops_per_s'], u['op_latency_ms'], u['background_builds'])"
