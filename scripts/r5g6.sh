# flake rate of the TP=8 group native loop case (separate processes, stop at the first failure)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread "tests/test_group_native_loop_gpu.py::test_group_native_loop_matches_python_lockstep[8]" -m gpu > gpurun_out/r5g6_$i.log 2>&1; rc=$?; echo "run $i rc=$rc"; tail -2 gpurun_out/r5g6_$i.log; [ $rc -eq 0 ] || exit $rc
done
