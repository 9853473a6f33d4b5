#!/bin/bash
# Round 6: Mixtral-8x7B EP=4 all-to-all (DP attention) group on virtual ranks (all four rank
# processes on the box's one GPU), served through the cluster: native group loop vs the
# Python lockstep loop (compares the loops, not multi-GPU speed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp P2P_CAR_TIMEOUT_MS=30000 P2P_QA_TIMEOUT_MS=30000
TAG=${TAG:-r6x}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
step 500 ${TAG}_a2a_native.log python bench/serve_bench.py --model mixtral-8x7b --gpus 4 --ep 4 --ep-mode a2a --virtual 1 --peers 8 --requests 4 --loop native --kv-pages 512
step 500 ${TAG}_a2a_python.log python bench/serve_bench.py --model mixtral-8x7b --gpus 4 --ep 4 --ep-mode a2a --virtual 1 --peers 8 --requests 4 --loop python --kv-pages 512
