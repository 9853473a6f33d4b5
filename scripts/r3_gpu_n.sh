#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qkv_attn_gpu.py > $O/qa_test.log 2>&1
rc=$?; echo "qa test rc=$rc"; grep -h "PASSED\|FAILED\|Error" $O/qa_test.log | head -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench/qkv_attn_bench.py > $O/qa_bench.jsonl 2> $O/qa_bench.err; echo "rc=$?"; cat $O/qa_bench.jsonl
