#!/bin/bash
# rocprofv3 kernel stats of the headline bench at 1 and 8 peers per GPU (llama3.1-8B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for P in ${PEERS:-1 8}; do
  mkdir -p gpurun_out/prof_p$P
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p$P -o run \
    -- python3 bench.py --steps 3 --warmup 1 --peers $P > gpurun_out/prof_p$P/bench.log 2>&1
  rc=$?; echo "peers=$P rocprof rc=$rc"; tail -1 gpurun_out/prof_p$P/bench.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
find gpurun_out -name "*kernel_stats.csv" | head
