#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3q
mkdir -p $O
run() { timeout -k 10 200 python -u bench/serve_bench.py --peers $1 --requests $((256 / $1)) > $O/$2.jsonl 2> $O/$2.err || exit 1; python -c "
import json; d=json.loads(open('$O/$2.jsonl').read()); print('$2', d['value'], d['ttft_p50_ms'], d['ttft_p99_ms'], d['queue_p50_ms'], d['queue_p99_ms'], d['mean_batch'], d['engine_time_s'])"; }
run 32 p32_default
ENGINE_ADMIT_WAIT_US=2000 run 32 p32_wait2ms
run 8 p8_default
