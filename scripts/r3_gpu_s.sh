#!/bin/bash
# round 3 session 2: kernel numerics after the epilogue-batching change, mid-M family
# timings, headline bench.  Each GPU step has its own limit; a failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels_test.log 2>&1 || { tail -30 $O/kernels_test.log; exit 1; }
tail -2 $O/kernels_test.log
timeout -k 10 400 python -u bench/wide_bench.py ${WB_M:-8 44} > $O/wide_bench.jsonl 2> $O/wide_bench.err || { tail -5 $O/wide_bench.err; exit 1; }
cat $O/wide_bench.jsonl
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -n "${AFRAG:-}" ]; then
  timeout -k 10 400 python -u bench/afrag_probe.py ${AFRAG_M:-8 44} > $O/afrag_probe.jsonl 2> $O/afrag_probe.err || { tail -5 $O/afrag_probe.err; exit 1; }
  cat $O/afrag_probe.jsonl
fi
