#!/bin/bash
# Round 6, third GPU session: wide16 with one chunk ahead (numerics + sweep + stamps), the
# 16-wave skinny GEMV (numerics), bench with an online re-tune, fused all-reduce engines
# (TP=4 then TP=8, each its own step, virtual ranks), then this round's feature tests + smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 400 r6c_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "wide or 16_waves or skinny"
WIDE_OTHERS=0 WIDE_SPLITS=0,4,5,6,8 step 300 r6c_wide.jsonl python bench/wide_bench.py 48
PROBE_NW=16 PROBE_SPLITS=0 step 200 r6c_stamps16.jsonl python bench/wide_stamp_probe.py
P2P_AUTOTUNE_TABLE=0 step 300 r6c_bench_tuned.log python bench.py --steps 20 --warmup 5
step 300 r6c_far4.log python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_world8_gpu.py -k "dense-tp-4"
