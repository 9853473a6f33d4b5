#!/bin/bash
# 70B TP=8 rank proxy: fused vs unfused row-parallel all-reduce, and a rocprofv3 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
P2P_TP_FUSED_AR=0 timeout -k 10 400 python -u bench/tp_rank_proxy.py --steps 5 --warmup 2 > $O/proxy_unfused.jsonl 2> $O/proxy_unfused.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench/tp_rank_proxy.py --steps 3 --warmup 1 > $O/proxy_prof.jsonl 2> $O/proxy_prof.err
echo "rc=$?"; cat $O/proxy_unfused.jsonl $O/proxy_prof.jsonl | grep decode_ms
find $O/prof -name "*stats*"
