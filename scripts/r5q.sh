set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k tall > gpurun_out/r5q_test.log 2>&1; rc=$?; tail -15 gpurun_out/r5q_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/prefill_gemm_bench.py --M 96 128 160 192 288 352 384 --gemms gate_up --only v2_auto v2_256x256_phased v2_192x128 > gpurun_out/r5q_prefill.jsonl 2>&1; rc=$?; grep -E "tall|hipblaslt|v2_auto" gpurun_out/r5q_prefill.jsonl; exit $rc
