#!/bin/bash
# round 3 session 2: full GPU tier, then the TTFT anatomy (wall vs GPU, kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench/ttft_breakdown.py --iters 20 > $O/ttft.json 2> $O/ttft.err || { tail -5 $O/ttft.err; exit 1; }
cat $O/ttft.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench/ttft_breakdown.py --iters 5 > $O/ttft_prof.log 2>&1 || { tail -5 $O/ttft_prof.log; exit 1; }
find $O/prof -name "*.csv" | head
