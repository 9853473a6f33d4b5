#!/bin/bash
# Round 6: where the qkv+attention tail goes at 8B decode -- producers only, hand-off only,
# hand-off after the consumers' K/V pages landed, full kernel (default and 2-key-wave launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6z}
timeout -k 10 300 python -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_qkv_attn_gpu.py > gpurun_out/${TAG}_qa_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_qa_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_qa_tests.log
timeout -k 10 400 python bench/qkv_attn_bench.py > gpurun_out/${TAG}_qa_bench.log 2>&1
rc=$?; grep '"shape"' gpurun_out/${TAG}_qa_bench.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], d['M'], {k:v for k,v in d.items() if k.startswith('fused') and 'ks' not in k or k in ('qkv_only','two_kernels')})"
exit $rc
