#!/bin/bash
# Round 6: native-loop GPU tests after the staging-slot fix, the TP=8 group determinism
# probe (each loop twice), then the 8-peer prompt chunk profile (scripts/r6_probe10.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6m}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 600 ${TAG}_loop.log python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_native_loop_gpu.py tests/test_group_native_loop_gpu.py -k "not graph_matches_eager"
step 600 ${TAG}_det8.log python -u bench/group_determinism.py --world 8
tail -4 gpurun_out/${TAG}_det8.log
TAG=$TAG bash scripts/r6_probe10.sh
