set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1050 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r5k_pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r5k_pytest_gpu.log; exit $rc
