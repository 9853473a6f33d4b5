# Granule split-K seam in the wide mid-M GEMM: kernel tests, per-phase stamps, TTFT.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r5s}
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 400 ${T}_test.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wide or midm" &&
run 300 ${T}_stamp.jsonl python bench/wide_stamp_probe.py &&
run 300 ${T}_ttft.log python bench/ttft_breakdown.py --message 4 --pages 2
