#!/bin/bash
# Round 6, second GPU session: the 16-wave wide kernel -- numerics (every epilogue vs fp32,
# both wave counts), the per-projection sweep at the prompt size, the headline bench with an
# online re-tune (the new candidates); then the fused all-reduce with the co-resident grid cap
# (per-kernel world 8, and the full-width TP=8 / TP=4 engines on virtual ranks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 400 r6b_widetests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k wide
WIDE_OTHERS=0 WIDE_SPLITS=0,2,3,4,5,6,8 step 300 r6b_wide.jsonl python bench/wide_bench.py 48
P2P_AUTOTUNE_TABLE=0 step 300 r6b_bench_tuned.log python bench.py --steps 20 --warmup 5
step 500 r6b_far.log python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_fused_ar_gpu.py tests/test_world8_gpu.py -k "fused or dense"
