# Bisect: world-8 TP=4 virtual-rank case on the pre-granule-seam wide kernel.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_world8_gpu.py::test_world8_virtual_ranks_full_width[dense-tp-4-env1]" -m gpu > gpurun_out/r5g4.log 2>&1; rc=$?; tail -3 gpurun_out/r5g4.log; exit $rc
