#!/bin/bash
# Round 6: the world-8 sampled-reply nondeterminism in the GPU test file's order (worlds 2 and
# 4 first), native loop 3x + Python loop once; then the same with one-step group graphs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6ab}
timeout -k 10 500 python -u bench/group_determinism.py --sequence 3 > gpurun_out/${TAG}_seq.log 2>&1 || { tail -5 gpurun_out/${TAG}_seq.log; exit 1; }
grep -E "^native|^python|sequence" gpurun_out/${TAG}_seq.log
P2P_GROUP_GRAPH_STEPS=1 timeout -k 10 500 python -u bench/group_determinism.py --sequence 3 > gpurun_out/${TAG}_seq_steps1.log 2>&1 || { tail -5 gpurun_out/${TAG}_seq_steps1.log; exit 1; }
grep -E "^native|^python|sequence" gpurun_out/${TAG}_seq_steps1.log
