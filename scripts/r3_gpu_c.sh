#!/bin/bash
# world-8 virtual-rank engine variants (fused / unfused / capped waves / world 4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_world8_gpu.py > $O/world8.log 2>&1
echo "rc=$?"
grep -h "PASSED\|FAILED\|passed\|failed\|tokens \[" $O/world8.log | head -20
