#!/bin/bash
# Round 6: follower collective-timeout status bit on the GPU, plus the group native-loop
# regressions (TP 2/4/8, follower fault, EP a2a).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6aa}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu -rx \
  tests/test_group_native_loop_gpu.py tests/test_native_loop_gpu.py > gpurun_out/${TAG}_loop.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|XFAIL|SKIPPED|ERROR" gpurun_out/${TAG}_loop.log | cut -c1-160 | tail -25; exit $rc
