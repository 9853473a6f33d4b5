#!/bin/bash
# full GPU tier + smoke + serving baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 $O/smoke.log
timeout -k 10 300 python -u bench/serve_bench.py --peers 8 --requests 8 > $O/serve8.jsonl 2> $O/serve8.err
echo "serve8 rc=$?"; cat $O/serve8.jsonl
timeout -k 10 300 python -u bench/serve_bench.py --peers 32 --requests 4 > $O/serve32.jsonl 2> $O/serve32.err
echo "serve32 rc=$?"; cat $O/serve32.jsonl
