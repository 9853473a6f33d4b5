# A/B: wide mid-M K slices on k-step vs chunk boundaries (P2P_WIDE_KSTEP), prompt-chunk TTFT.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-400; return $rc; }
run 400 r5x_test.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wide" &&
for i in 1 2; do
  P2P_WIDE_KSTEP=1 run 300 r5x_ttft_k1_$i.log python bench/ttft_breakdown.py --message 4 --pages 2 &&
  P2P_WIDE_KSTEP=0 run 300 r5x_ttft_k0_$i.log python bench/ttft_breakdown.py --message 4 --pages 2 || exit 1
done
