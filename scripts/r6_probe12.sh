#!/bin/bash
# Round 6, VERDICT r5 item 2: the persistent decode engine generalised to the 70B TP=8 rank
# shapes (k-ranges under the prefetch credit / not a multiple of the batch, more workgroups
# than qkv half groups): numerics vs the per-layer launches, then engine vs launches at the
# shard shapes (3584-column ffn and the 3072 / 4096 bracket) and at 8B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6n}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 400 ${TAG}_detests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_decode_engine_gpu.py
step 300 ${TAG}_de3584.log python bench/decode_engine_bench.py --tp8-shard --iters 100
step 300 ${TAG}_de4096.log python bench/decode_engine_bench.py --tp8-shard --ffn 4096 --iters 100
step 300 ${TAG}_de3072.log python bench/decode_engine_bench.py --tp8-shard --ffn 3072 --iters 100
step 300 ${TAG}_de8b.log python bench/decode_engine_bench.py --iters 100
step 300 ${TAG}_de3584_trace.log python bench/decode_engine_bench.py --tp8-shard --iters 50 --trace
