#!/bin/bash
# Round 6: fused all-reduce at TP=8 on virtual ranks with one hardware queue per rank process
# (hypothesis: 8 processes x 4 queues oversubscribe the device's mapped queues), then the
# serving-path GPU tests and the graph-vs-eager TP prefill test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6e}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
# a plain test failure (rc 1: a bounded collective wait, no GPU fault) does not stop the run
echo "== ${TAG}_far8q1.log $(date +%T)"
GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-8-env0" > gpurun_out/${TAG}_far8q1.log 2>&1
rc=$?; echo "far8q1 rc=$rc"; tail -3 gpurun_out/${TAG}_far8q1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=$TAG bash scripts/r6_gpu_tests.sh || exit $?
step 600 ${TAG}_forms.log python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "graph_matches_eager"
