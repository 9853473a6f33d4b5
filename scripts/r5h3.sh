# 8-peer batched prefill with the 192x256 gate_up pick: TTFT breakdown, gate_up at 288-384 rows, bench --peers 8.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-300; return $rc; }
run 300 r5h3_ttft8.log python bench/ttft_breakdown.py --message 4 --pages 2 --peers 8 &&
run 300 r5h3_gu.jsonl python bench/prefill_gemm_bench.py --M 288 320 352 384 --gemms gate_up --only v2_auto &&
run 600 r5h3_bench8.log python bench.py --peers 8 --steps 10 --warmup 3
