cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_multidev.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
GPC_COMPACT_DEBUG=1 bash tools/c5_long.sh r05c 3500 2>&1 | tail -5
