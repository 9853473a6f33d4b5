#!/bin/bash
# Round 6, VERDICT r5 item 4: the EP all-to-all (DP-attention) virtual group on the native
# loop vs the Python lockstep loop, then the native-loop regressions (single GPU + TP groups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6p}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 500 ${TAG}_a2a.log python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "a2a"
step 700 ${TAG}_loop.log python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_native_loop_gpu.py tests/test_group_native_loop_gpu.py -k "not a2a"
