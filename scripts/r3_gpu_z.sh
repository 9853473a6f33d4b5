#!/bin/bash
# round 3 session 2: the other models on one GPU with the current kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --steps 3 --warmup 1 > $O/mixtral_p1.json 2> $O/mixtral_p1.err || { tail -5 $O/mixtral_p1.err; exit 1; }
tail -1 $O/mixtral_p1.json
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --peers 8 --steps 3 --warmup 1 > $O/mixtral_p8.json 2> $O/mixtral_p8.err || { tail -5 $O/mixtral_p8.err; exit 1; }
tail -1 $O/mixtral_p8.json
timeout -k 10 500 python -u bench.py --model llama3.1-70b --steps 2 --warmup 1 > $O/l70_p1.json 2> $O/l70_p1.err || { tail -5 $O/l70_p1.err; exit 1; }
tail -1 $O/l70_p1.json
timeout -k 10 300 python -u bench/serve_bench.py --peers 8 --requests 32 > $O/serve_p8.json 2> $O/serve_p8.err || { tail -5 $O/serve_p8.err; exit 1; }
tail -1 $O/serve_p8.json
