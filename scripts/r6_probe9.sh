#!/bin/bash
# Round 6: the TP=8 group's sampled reply (native loop vs Python lockstep) with the fused
# all-reduce epilogue on and off, and the 8-peer bench (384-row batched prefill).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6j}
run_nf() {  # a plain test failure (rc 1) does not stop the run
  local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?
  echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
P2P_TP_FUSED_AR=0 run_nf 400 ${TAG}_group8_far0.log python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "matches_python_lockstep and 8"
P2P_TP_FUSED_AR=1 run_nf 400 ${TAG}_group8_far1.log python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "matches_python_lockstep and 8"
run_nf 400 ${TAG}_peers8.log python bench.py --peers 8 --steps 10 --warmup 3
