#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_world8_gpu.py tests/test_fused_ar_gpu.py tests/test_parallel_gpu.py > $O/tests.log 2>&1
echo "tests rc=$?"
grep -h "PASSED\|FAILED\|passed\|failed" $O/tests.log | head -30
timeout -k 10 400 python -u bench/tp_rank_proxy.py --steps 5 --warmup 2 > $O/proxy70b.jsonl 2> $O/proxy70b.err
echo "proxy rc=$?"; cat $O/proxy70b.jsonl; tail -3 $O/proxy70b.err
