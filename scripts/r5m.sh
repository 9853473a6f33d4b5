set -o pipefail
mkdir -p gpurun_out/prof8
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python bench.py --peers 8 --steps 10 --warmup 3 > gpurun_out/r5m_bench8.log 2>&1; rc=$?; tail -1 gpurun_out/r5m_bench8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run -- python3 bench.py --peers 8 --steps 3 --warmup 1 > gpurun_out/r5m_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; find gpurun_out/prof8 -name "*.db" -o -name "*stats*" | head
