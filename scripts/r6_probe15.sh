#!/bin/bash
# Round 6: batch-1 residual GEMVs load their residual before the weight stream (skinny
# EPI_RESID / EPI_AR): numerics, then the headline bench twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6q}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 600 ${TAG}_tests.log python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_fused_ar_gpu.py -k "skinny or fused or resid or far"
step 400 ${TAG}_bench1.log python bench.py --steps 20 --warmup 5
step 400 ${TAG}_bench2.log python bench.py --steps 20 --warmup 5
