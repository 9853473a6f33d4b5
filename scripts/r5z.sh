# BD tiles of the prefill GEMM: correctness (tiled tests) and batched-prompt timings vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 500 r5z_test.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tiled" &&
run 600 r5z_prefill.jsonl python bench/prefill_gemm_bench.py --M 160 192 256 384 512 --only v2_auto bd_192x256 bd_128x256 bd_192x128 bd_128x128 bd_192x256_s1 bd_128x256_s1
