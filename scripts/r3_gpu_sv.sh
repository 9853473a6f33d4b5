#!/bin/bash
# serving burst policy: prefill budget per step x prefill-first, 32 and 8 peers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3sv
mkdir -p $O
run() {  # peers max_prefill prefill_first tag
  ENGINE_PREFILL_FIRST=$3 timeout -k 10 240 python -u bench/serve_bench.py --peers $1 --requests $((256 / $1)) --max-prefill $2 > $O/$4.json 2> $O/$4.err || { tail -3 $O/$4.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/$4.json').read().strip().splitlines()[-1]); print('$4', d['value'], d['ttft_p50_ms'], d['ttft_p99_ms'], d['queue_p99_ms'])"
}
run 32 1024 0 p32_b1024_pf0
run 32 1024 1 p32_b1024_pf1
run 32 2048 1 p32_b2048_pf1
run 8 1024 1 p8_b1024_pf1
run 8 2048 1 p8_b2048_pf1
