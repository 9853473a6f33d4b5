#!/bin/bash
# round 3 session 2: headline bench (driver form), rocprofv3 stats of it, 70B TP=8 rank proxy,
# 8-peer static batch, continuous batching
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u bench/tp_rank_proxy.py > $O/tp8_proxy.json 2> $O/tp8_proxy.err || { tail -5 $O/tp8_proxy.err; exit 1; }
cat $O/tp8_proxy.json
timeout -k 10 300 python -u bench.py --peers 8 --steps 10 --warmup 3 > $O/bench_p8.json 2> $O/bench_p8.err || { tail -5 $O/bench_p8.err; exit 1; }
cat $O/bench_p8.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof_bench.log 2>&1 || { tail -5 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log
