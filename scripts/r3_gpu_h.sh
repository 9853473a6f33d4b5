#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
for p in 8 32; do
timeout -k 10 300 python -u bench/serve_bench.py --peers $p --requests $((256 / p)) > $O/serve$p.jsonl 2> $O/serve$p.err || exit 1
cat $O/serve$p.jsonl
done
ENGINE_ADMIT_WAIT_US=0 timeout -k 10 300 python -u bench/serve_bench.py --peers 8 --requests 32 > $O/serve8_nowait.jsonl 2> $O/serve8_nowait.err
cat $O/serve8_nowait.jsonl
