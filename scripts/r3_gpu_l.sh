#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/qa -o run -- python3 bench.py --steps 3 --warmup 1 > $O/qa.log 2>&1; echo "rc=$?"
export P2P_QKV_ATTN=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/noqa -o run -- python3 bench.py --steps 3 --warmup 1 > $O/noqa.log 2>&1; echo "rc=$?"
