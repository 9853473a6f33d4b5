#!/bin/bash
# Round 6 end-of-session: smoke, serving with >= 256 timed requests per config (p99 over a
# real sample), the 8-peer static batch and the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6u}
step() { local lim=$1 log=$2; shift 2; echo "== $log $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step 300 ${TAG}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 ${TAG}_serve8.log python bench/serve_bench.py --peers 8 --requests 32
step 400 ${TAG}_serve32.log python bench/serve_bench.py --peers 32 --requests 8
step 300 ${TAG}_peers8.log python bench.py --peers 8 --steps 10 --warmup 3
step 300 ${TAG}_bench.log python bench.py --steps 20 --warmup 5
