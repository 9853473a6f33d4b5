set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "tiled" --timeout 120 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; tail -3 gpurun_out/t_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/midm_split_bench.py > gpurun_out/midm_split.jsonl 2>&1
