#!/bin/bash
# Round 6: fused all-reduce on co-resident virtual ranks, then this round's
# serving-path GPU tests (native BPE, cluster request path, follower faults) and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6d}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 400 ${TAG}_far4.log python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-4"
step 400 ${TAG}_far8.log python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-8-env0"
TAG=$TAG bash scripts/r6_gpu_tests.sh || exit $?
step 600 ${TAG}_forms.log python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "graph_matches_eager"
