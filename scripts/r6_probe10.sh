#!/bin/bash
# Round 6: the 8-peer prompt chunk (352 rows -> 384-row bucket): wall vs GPU time, then the
# per-kernel table under rocprofv3 (kernel trace + stats only).
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6l}
timeout -k 10 300 python bench/ttft_breakdown.py --message 4 --pages 2 --peers 8 --iters 20 > gpurun_out/${TAG}_ttft8.log 2>&1 || exit $?
tail -2 gpurun_out/${TAG}_ttft8.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof8 -o run -- python3 "$GRAFT_REPO_ROOT/bench/ttft_breakdown.py" --message 4 --pages 2 --peers 8 --iters 20 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
db=$(find /tmp/prof8 -name '*results.db' | head -1)
python3 scripts/kstats_db.py "$db" 24 > gpurun_out/${TAG}_kstats8.md && cat gpurun_out/${TAG}_kstats8.md
