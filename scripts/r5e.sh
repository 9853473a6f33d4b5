set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chat_integration.py -m gpu -k in_process tests/test_native_loop_gpu.py > gpurun_out/r5e_test.log 2>&1; rc=$?; tail -15 gpurun_out/r5e_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/e2e_suggest_bench.py > gpurun_out/r5e_e2e.log 2>&1; rc=$?; tail -2 gpurun_out/r5e_e2e.log; exit $rc
