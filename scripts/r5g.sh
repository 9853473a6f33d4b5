set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_group_native_loop_gpu.py tests/test_cluster_gpu.py tests/test_world8_gpu.py > gpurun_out/r5g_test.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r5g_test.log | tail -30; exit $rc
