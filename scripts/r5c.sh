set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wide" > gpurun_out/r5c_test.log 2>&1; rc=$?; tail -3 gpurun_out/r5c_test.log; [ $rc -eq 0 ] || exit $rc
PROBE_SPLITS=0 timeout -k 10 300 python bench/wide_stamp_probe.py > gpurun_out/r5c_stamp.jsonl 2>&1 && cat gpurun_out/r5c_stamp.jsonl &&
timeout -k 10 300 python bench.py > gpurun_out/r5c_bench.log 2>&1 && tail -1 gpurun_out/r5c_bench.log
