set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qkv_attn_gpu.py > gpurun_out/r5o_test.log 2>&1; rc=$?; tail -15 gpurun_out/r5o_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/qkv_attn_bench.py > gpurun_out/r5o_qa.jsonl 2>&1; rc=$?; cat gpurun_out/r5o_qa.jsonl | grep shape; exit $rc
