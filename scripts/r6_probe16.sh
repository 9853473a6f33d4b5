#!/bin/bash
# Round 6: re-tune the pinned launch tables against the round-6 kernels (16-wave wide GEMM,
# early-residual GEMVs): 8B and the 70B TP=8 rank shard.  The JSON lines land in gpurun_out/
# and are written to engine/tuned/ on the builder.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6r}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 "gpurun_out/$log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step 500 ${TAG}_tune8b_a.log python -m p2p_llm_chat_go_amd.engine.autotune --model llama3.1-8b
step 500 ${TAG}_tune8b_b.log python -m p2p_llm_chat_go_amd.engine.autotune --model llama3.1-8b
step 500 ${TAG}_tune70b.log python -m p2p_llm_chat_go_amd.engine.autotune --model llama3.1-70b --tp 8 --batch 1,2,4,8,16,48,64
