#!/bin/bash
# Round 6 end-of-session GPU tier, in the driver's form (one pytest process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6t}
timeout -k 10 1080 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread -rx > gpurun_out/${TAG}_gpu_tier.log 2>&1
rc=$?
echo "gpu tier rc=$rc"; tail -6 gpurun_out/${TAG}_gpu_tier.log
exit $rc
