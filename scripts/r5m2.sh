# Other model families on the round-5 tree: Mixtral-8x7B (1 and 8 peers) and llama3.1-70B TP=1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-300; return $rc; }
run 500 r5m2_mixtral1.log python bench.py --model mixtral-8x7b --steps 3 --warmup 1 &&
run 500 r5m2_mixtral8.log python bench.py --model mixtral-8x7b --peers 8 --steps 3 --warmup 1 &&
run 600 r5m2_70b.log python bench.py --model llama3.1-70b --steps 3 --warmup 1
