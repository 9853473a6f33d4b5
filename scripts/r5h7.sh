# split-K fault word shared by tiled / wide kernels and checked by the native loop; serving refresh
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-400; return $rc; }
run 600 r5h7_test.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_loop_gpu.py tests/test_kernels_gpu.py tests/test_engine.py -m gpu -k "native_loop or tiled or wide or split or prefill_graph" &&
run 400 r5h7_serve8.log python bench/serve_bench.py --peers 8 --requests 6 &&
run 500 r5h7_serve32.log python bench/serve_bench.py --peers 32 --requests 4 &&
run 300 r5h7_prefill288.jsonl python bench/prefill_gemm_bench.py --cold --M 288 --only v2_auto
