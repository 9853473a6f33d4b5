#!/bin/bash
# Round 6 session 2: kernel table of the 8-peer prompt chunk (384-row bucket) on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$PWD
TAG=${TAG:-r6p8p}
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof8p -o run -- python3 "$R/bench/ttft_breakdown.py" --message 4 --pages 2 --peers 8 --iters 20 > "$R/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
cd "$R"
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-300
db=$(find /tmp/prof8p -name '*results.db' | head -1)
python3 scripts/kstats_db.py "$db" 24 > gpurun_out/${TAG}_kstats.md && cat gpurun_out/${TAG}_kstats.md
