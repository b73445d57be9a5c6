cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
for c in C2g C2 C3 C1; do
timeout -k 10 900 python -u bench.py --config $c --no-cpu-baseline --no-traffic --steps 20 > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_by_launch'], d['parity']['mismatches'], d['config']['image_mb'])" $O/$c.json $c
done
