#!/bin/bash
# Round 3, GPU call A: fused all-reduce epilogue + world-8 virtual ranks + 70B TP=8 rank proxy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import torch; print('cuda', torch.cuda.is_available(), flush=True)" &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fused_ar_gpu.py > $O/fused_ar.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_world8_gpu.py tests/test_parallel_gpu.py > $O/world8.log 2>&1 &&
timeout -k 10 400 python -u bench/tp_rank_proxy.py --steps 5 --warmup 2 > $O/proxy70b.jsonl 2> $O/proxy70b.err &&
echo ALL_OK
rc=$?
tail -5 $O/*.log $O/proxy70b.jsonl 2>/dev/null
exit $rc
