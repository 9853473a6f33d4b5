# 192x256 prefill tile: correctness, then batched-prompt timings vs the current picks and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 "gpurun_out/$log"; return $rc; }
run 500 r5h2_test.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tiled" &&
run 600 r5h2_prefill.jsonl python bench/prefill_gemm_bench.py --M 192 256 384 512 --only v2_auto v2_256x256_phased v2_192x256 v2_192x256_s1 v2_192x256_s2
