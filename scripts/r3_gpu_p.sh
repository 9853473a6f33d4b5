#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3p
mkdir -p $O
for p in 8 32; do
timeout -k 10 300 python -u bench/serve_bench.py --peers $p --requests $((256 / p)) > $O/serve$p.jsonl 2> $O/serve$p.err || exit 1
cat $O/serve$p.jsonl
done
timeout -k 10 300 python -u bench/car_crossover.py --world 8 > $O/crossover8.jsonl 2> $O/crossover8.err; echo "xover rc=$?"; cat $O/crossover8.jsonl
timeout -k 10 300 python -u bench/car_crossover.py --world 4 > $O/crossover4.jsonl 2> $O/crossover4.err; echo "xover4 rc=$?"; cat $O/crossover4.jsonl
