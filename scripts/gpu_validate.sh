# End-of-session GPU validation: virtual-rank / group-loop / wide-kernel tests, the rest of the
# GPU tier, smoke and the headline bench (logs: gpurun_out/r5g3_*).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 500 r5g3_world8.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_world8_gpu.py tests/test_group_native_loop_gpu.py tests/test_kernels_gpu.py -k "world8 or group_native or wide" -m gpu &&
run 700 r5g3_rest.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "not world8 and not group_native" &&
run 300 r5g3_smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
run 600 r5g3_bench.log python bench.py --steps 20 --warmup 5
