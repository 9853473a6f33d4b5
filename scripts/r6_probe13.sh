#!/bin/bash
# Round 6: the decode engine's per-phase stamps at the 70B TP=8 shard shapes, and the rank
# proxy's kernel table (rocprofv3 kernel trace + stats only).
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6o}
timeout -k 10 300 python bench/decode_engine_bench.py --tp8-shard --iters 50 --trace > gpurun_out/${TAG}_de_trace.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_de_trace.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof70 -o run -- python3 "$GRAFT_REPO_ROOT/bench/tp_rank_proxy.py" --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_proxy_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
tail -1 gpurun_out/${TAG}_proxy_prof.log
db=$(find /tmp/prof70 -name '*results.db' | head -1)
python3 scripts/kstats_db.py "$db" 30 > gpurun_out/${TAG}_proxy_kstats.md && head -40 gpurun_out/${TAG}_proxy_kstats.md
