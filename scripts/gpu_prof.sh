#!/bin/bash
# Kernel-level profile of the headline bench (rocprofv3 kernel trace + stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
