#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/ttft_breakdown.py --iters 30 > $O/ttft.jsonl 2> $O/ttft.err; echo rc=$?; cat $O/ttft.jsonl
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.jsonl 2> $O/bench.err; echo rc=$?; cat $O/bench.jsonl | cut -c1-400
