#!/bin/bash
# Quick GPU check: selected test files, then the default bench line (tools/gpu_session.sh runs the full set).
#   tools/gpu_quick.sh TAG "tests/test_a.py tests/test_b.py" [bench args...]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}; TESTS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
if [ -n "$TESTS" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
  tail -4 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench $(date +%T)"
timeout -k 10 600 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
