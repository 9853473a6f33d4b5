#!/bin/bash
# Round 6, VERDICT r5 item 2: the persistent whole-step decode engine at the llama3.1-70B
# TP=8 rank shapes, bracketed by ffn widths its 1024-column unit divides (4096 above the
# real 3584, 3072 below), against the per-layer launches at the same shapes; then the rank
# proxy itself (current tree, pinned table and an online re-tune).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6i}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
echo "== ${TAG}_far8.log $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-8-env0" > gpurun_out/${TAG}_far8.log 2>&1
rc=$?; echo "far8 rc=$rc"; tail -3 gpurun_out/${TAG}_far8.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step 300 ${TAG}_de4096.log python bench/decode_engine_bench.py --tp8-shard --ffn 4096 --iters 100
step 300 ${TAG}_de3072.log python bench/decode_engine_bench.py --tp8-shard --ffn 3072 --iters 100
step 300 ${TAG}_de3584.log python bench/decode_engine_bench.py --tp8-shard --iters 100
step 400 ${TAG}_proxy.log python bench/tp_rank_proxy.py --steps 10 --warmup 3
