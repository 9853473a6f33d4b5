# continuous batching through the native loop after the granule seam: 8 and 32 peers
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-400; return $rc; }
run 400 r5h6_serve8.log python bench/serve_bench.py --peers 8 --requests 6 &&
run 500 r5h6_serve32.log python bench/serve_bench.py --peers 32 --requests 4
run 300 r5h6_prefill288.jsonl python bench/prefill_gemm_bench.py --cold --M 288 --only v2_auto
