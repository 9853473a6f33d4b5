#!/bin/bash
# round 3 session 2: one-m-tile 384/448-row prefill tiles: tiled tests, sweep, 8-peer bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "tiled" --timeout 120 --timeout-method thread > $O/tiled_test.log 2>&1 || { tail -30 $O/tiled_test.log; exit 1; }
tail -1 $O/tiled_test.log
timeout -k 10 600 python -u bench/prefill_gemm_bench.py --M 352 400 440 --only v2_auto v2_256x256_phased v2_320x128 v2_384x128 v2_448x128 v2_128x128 > $O/prefill_sweep.jsonl 2> $O/prefill_sweep.err || { tail -5 $O/prefill_sweep.err; exit 1; }
timeout -k 10 300 python -u bench.py --peers 8 --steps 5 --warmup 2 > $O/bench_p8.json 2> $O/bench_p8.err || { tail -5 $O/bench_p8.err; exit 1; }
cat $O/bench_p8.json
