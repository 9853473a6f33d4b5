#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qkv_attn_gpu.py > $O/qa_test.log 2>&1
rc=$?; echo "qa test rc=$rc"; grep -h "PASSED\|FAILED\|Error\|assert" $O/qa_test.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_qa.jsonl 2> $O/bench_qa.err; echo "bench rc=$?"
P2P_QKV_ATTN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_noqa.jsonl 2> $O/bench_noqa.err; echo "bench0 rc=$?"
python -c "
import json
for f in ('bench_qa','bench_noqa'):
    d=json.loads(open('$O/'+f+'.jsonl').read().strip().splitlines()[-1]); print(f, d['value'], d['ttft_p50_ms'], d['ms_per_step'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine.py tests/test_hf_parity.py tests/test_parallel_gpu.py tests/test_world8_gpu.py > $O/engine_tests.log 2>&1; echo "engine tests rc=$?"; tail -3 $O/engine_tests.log
