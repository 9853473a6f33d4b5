#!/bin/bash
# Round 6, session 2: the GPU commands behind the session's profiles (one MI355X).
#   profiles/r6_mall_probe.jsonl             Infinity-Cache warm vs cold projections
#   profiles/r6_lmhead_probe_*.jsonl         greedy LM head: argmax vs fp32 epilogue per code
#   profiles/r6_gemv_codes_probe.jsonl       decode GEMVs at every launch code + tiny-kernel gap
#   profiles/r6_prefill_gemm_*_cold*.jsonl   prefill GEMM tile / split sweeps (96-512 rows)
#   profiles/r6_models_1gpu.jsonl            Mixtral-8x7B (1 / 8 peers), 70B TP=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6s2}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step 240 ${TAG}_mall.jsonl python -u bench/mall_probe.py 1 48
step 240 ${TAG}_lmhead.jsonl python -u bench/lmhead_probe.py
step 300 ${TAG}_gemv_codes.jsonl python -u bench/gemv_codes_probe.py
step 600 ${TAG}_pgemm.jsonl python -u bench/prefill_gemm_bench.py --M 96 128 192 256 384 512 --cold
step 400 ${TAG}_mixtral1.log python -u bench.py --model mixtral-8x7b --steps 3 --warmup 1
step 400 ${TAG}_mixtral8.log python -u bench.py --model mixtral-8x7b --peers 8 --steps 3 --warmup 1
step 500 ${TAG}_70b1.log python -u bench.py --model llama3.1-70b --steps 3 --warmup 1
