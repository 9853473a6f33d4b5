#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err; echo "bench rc=$?"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --peers 8 > $O/bench_p8.jsonl 2> $O/bench_p8.err; echo "bench8 rc=$?"
timeout -k 10 400 python -u bench/tp_rank_proxy.py --steps 5 --warmup 2 > $O/proxy70b.jsonl 2> $O/proxy70b.err; echo "proxy rc=$?"
python - <<'PY'
import json
for f in ("bench", "bench_p8", "proxy70b"):
    d = json.loads([l for l in open("gpurun_out/r3o/%s.jsonl" % f) if l.startswith("{")][-1])
    print(f, {k: d.get(k) for k in ("value", "ttft_p50_ms", "ms_per_step", "decode_ms_per_token", "suggest_reply_tokens_per_sec")})
PY
