#!/bin/bash
# Round 6: rocprofv3 kernel table of the headline bench (kernel trace + stats only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$PWD
TAG=${TAG:-r6p8}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof8 -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/${TAG}_bench_prof.log" 2>&1 || exit $?
cd "$R"
tail -1 gpurun_out/${TAG}_bench_prof.log | cut -c1-300
db=$(find /tmp/prof8 -name '*results.db' | head -1)
python3 scripts/kstats_db.py "$db" 30 > gpurun_out/${TAG}_kstats.md && head -40 gpurun_out/${TAG}_kstats.md
