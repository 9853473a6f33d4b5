set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_qkv_attn_gpu.py tests/test_world8_gpu.py tests/test_group_native_loop_gpu.py > gpurun_out/r5p_test.log 2>&1; rc=$?; tail -3 gpurun_out/r5p_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/tp_rank_proxy.py > gpurun_out/r5p_proxy.log 2>&1; rc=$?; tail -1 gpurun_out/r5p_proxy.log; exit $rc
