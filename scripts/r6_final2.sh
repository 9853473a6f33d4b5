#!/bin/bash
# Round 6, end of session: the GPU tier in the driver's form (one pytest process), smoke and
# the headline bench on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6f2}
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread -rx > gpurun_out/${TAG}_gpu_tier.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tier.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
