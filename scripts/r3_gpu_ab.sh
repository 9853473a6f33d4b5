#!/bin/bash
# A/B of the fused qkv+attention producers' rope-table fetch (before / after the weight stream):
# kernel microbench, then the headline bench alternated twice per mode on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3ab
mkdir -p $O
for mode in 0 1; do
  P2P_QA_EARLY_ROPE=$mode timeout -k 10 300 python -u bench/qkv_attn_bench.py > $O/qa_$mode.jsonl 2> $O/qa_$mode.err || exit 1
  head -1 $O/qa_$mode.jsonl
done
for rep in 1 2; do
  for mode in 0 1; do
    P2P_QA_EARLY_ROPE=$mode timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_${mode}_$rep.json 2> $O/bench_${mode}_$rep.err || exit 1
    python -c "import json; d=json.loads(open('$O/bench_${mode}_$rep.json').read().strip().splitlines()[-1]); print('early=$mode rep=$rep', d['value'], d['ttft_p50_ms'])"
  done
done
