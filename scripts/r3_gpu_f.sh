#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_fused_ar_gpu.py "tests/test_world8_gpu.py::test_world8_virtual_ranks_full_width[dense-tp-8-env0]" > $O/tests.log 2>&1
echo "tests rc=$?"; grep -h "PASSED\|FAILED\|passed\|failed" $O/tests.log | head
timeout -k 10 300 python -u bench/tp_rank_proxy.py --steps 5 --warmup 2 > $O/proxy_fused.jsonl 2> $O/proxy_fused.err
echo "proxy rc=$?"; grep -o '"decode_ms_per_token": [0-9.]*\|"ttft_p50_ms": [0-9.]*' $O/proxy_fused.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench/tp_rank_proxy.py --steps 2 --warmup 1 > $O/proxy_prof.jsonl 2> $O/proxy_prof.err
echo "prof rc=$?"
