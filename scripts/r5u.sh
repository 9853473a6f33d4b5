# Wide mid-M GEMM with k-step slices: kernel tests, stamps, TTFT, candidate re-check.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r5u}
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 400 ${T}_test.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wide or midm" &&
run 300 ${T}_stamp.jsonl python bench/wide_stamp_probe.py qkv o_proj down &&
run 300 ${T}_ttft.log python bench/ttft_breakdown.py --message 4 --pages 2 &&
run 500 ${T}_pick.jsonl python bench/midm_pick_check.py
