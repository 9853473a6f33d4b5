#!/bin/bash
# Round 6: the GPU tests of this round's features (native BPE / cluster request path through
# the C++ node, follower fault reporting, smoke with greedy tokens vs the fp32 oracle), one
# pytest process, then smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6b}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 900 ${TAG}_tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_chat_integration.py tests/test_group_native_loop_gpu.py -k "in_process or follower_fault or matches_python_lockstep"
step 300 ${TAG}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
