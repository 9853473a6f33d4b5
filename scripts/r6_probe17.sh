#!/bin/bash
# Round 6: the headline bench and the 70B TP=8 rank proxy on the re-tuned pinned tables.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6s}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-420; [ $rc -eq 0 ] || exit $rc; }
step 400 ${TAG}_bench1.log python bench.py --steps 20 --warmup 5
step 400 ${TAG}_bench2.log python bench.py --steps 20 --warmup 5
step 400 ${TAG}_bench3.log python bench.py --steps 20 --warmup 5
step 600 ${TAG}_proxy.log python bench/tp_rank_proxy.py
