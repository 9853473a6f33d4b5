#!/bin/bash
# world-8 co-scheduling probe: fused AR at world 8 with default / reduced HW queues per process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  "tests/test_fused_ar_gpu.py::test_fused_allreduce_epilogue_bit_identical[8]" > $O/w8_default.log 2>&1
echo "default rc=$?"
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  "tests/test_fused_ar_gpu.py::test_fused_allreduce_epilogue_bit_identical[8]" > $O/w8_q1.log 2>&1
echo "q1 rc=$?"
grep -h "timed out first\|passed\|failed" $O/*.log | head -20
