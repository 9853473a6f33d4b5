#!/bin/bash
# Round 6: determinism of the seeded sampled reply inside one TP=8 virtual-rank group
# (native loop, then Python loop), the request repeated 12 times in each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6y}
timeout -k 10 600 python -u bench/group_determinism.py --world 8 --repeat 12 > gpurun_out/${TAG}_rep8.log 2>&1
rc=$?; echo "rc=$rc"; grep '"loop"' gpurun_out/${TAG}_rep8.log; exit $rc
