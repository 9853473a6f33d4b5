#!/bin/bash
# Round 6, first GPU session: headline baseline on this tree, weight-stream probe, wide-kernel
# split sweep at the prompt size, then PMC passes (wide 48-row vs skinny batch-1 vs stream floor).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; [ $rc -eq 0 ] || exit $rc; }
step 300 r6a_bench.log python bench.py --steps 20 --warmup 5
step 300 r6a_stream.jsonl python bench/stream_probe.py
WIDE_OTHERS=0 WIDE_SPLITS=0,1,2,3,4,6,8 step 400 r6a_wide.jsonl python bench/wide_bench.py 48
bash scripts/pmc_passes.sh r6a_pmc bench/wide_pmc.py
