#!/bin/bash
# GPU validation sequence for one gpurun call: tests -> smoke -> bench.
# Each GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS=${STEPS:-tests,smoke,bench}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
