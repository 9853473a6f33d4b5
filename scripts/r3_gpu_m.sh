#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 300 python -u bench/qkv_attn_bench.py > $O/qa_bench.jsonl 2> $O/qa_bench.err; echo "rc=$?"; cat $O/qa_bench.jsonl; tail -3 $O/qa_bench.err
