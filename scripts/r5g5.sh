# group native loop (fused all-reduce at TP 2/4 on virtual ranks) after the world-8 TP=4 stalls
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_group_native_loop_gpu.py -m gpu > gpurun_out/r5g5.log 2>&1; rc=$?; tail -4 gpurun_out/r5g5.log; exit $rc
