#!/bin/bash
# Round 6: graph-vs-eager TP prefill logits (2/4/8 virtual ranks), the serving-path GPU tests,
# smoke, then the TP=8 fused all-reduce case with call-count reporting (a plain failure there
# does not stop the run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6h}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
echo "== ${TAG}_forms.log $(date +%T)"
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "graph_matches_eager" > gpurun_out/${TAG}_forms.log 2>&1
rc=$?; echo "forms rc=$rc"; tail -3 gpurun_out/${TAG}_forms.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== ${TAG}_far8.log $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-8-env0" > gpurun_out/${TAG}_far8.log 2>&1
rc=$?; echo "far8 rc=$rc"; tail -3 gpurun_out/${TAG}_far8.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step 900 ${TAG}_tests.log python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_chat_integration.py tests/test_group_native_loop_gpu.py -k "in_process or follower_fault"
step 300 ${TAG}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
