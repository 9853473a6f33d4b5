#!/bin/bash
# Round 6: the wide mid-M GEMM with every k-loop load / LDS read in asm (no compiler
# vmcnt(0) draining the ring pipeline): numerics, sweep, stamps (8 and 16 waves), bench with an
# online re-tune; then the serving-path GPU tests, the graph-vs-eager TP prefill test, and the
# TP=8 fused all-reduce case (a plain failure there does not stop the run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6f}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 400 ${TAG}_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "wide or 16_waves or skinny or tiled or midm"
WIDE_OTHERS=0 WIDE_SPLITS=0,4,6,8 step 300 ${TAG}_wide.jsonl python bench/wide_bench.py 48
PROBE_NW=8 PROBE_SPLITS=0 step 200 ${TAG}_stamps8.jsonl python bench/wide_stamp_probe.py
PROBE_NW=16 PROBE_SPLITS=0 step 200 ${TAG}_stamps16.jsonl python bench/wide_stamp_probe.py
P2P_AUTOTUNE_TABLE=0 step 300 ${TAG}_bench_tuned.log python bench.py --steps 20 --warmup 5
TAG=$TAG bash scripts/r6_gpu_tests.sh || exit $?
step 600 ${TAG}_forms.log python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_group_native_loop_gpu.py -k "graph_matches_eager"
echo "== ${TAG}_far8.log $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu \
  tests/test_world8_gpu.py -k "dense-tp-8-env0" > gpurun_out/${TAG}_far8.log 2>&1
rc=$?; echo "far8 rc=$rc"; tail -3 gpurun_out/${TAG}_far8.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
