#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_qkv_attn_gpu.py > $O/qa_test.log 2>&1
echo "rc=$?"; grep -h "PASSED\|FAILED\|AssertionError" $O/qa_test.log | head -30
