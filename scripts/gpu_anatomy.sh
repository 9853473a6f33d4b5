# Round-5 anatomy: TTFT breakdown, headline bench, rocprof kernel tables of the TTFT chunk,
# the headline bench and the 70B TP=8 rank proxy (SQLite outputs reduced to markdown on the
# box: the raw databases exceed what gpurun copies back).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r5r}
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 "gpurun_out/$log"; return $rc; }
prof() {  # prof <name> <timeout> <tokens> cmd...
  local name=$1 lim=$2 tok=$3; shift 3
  run "$lim" ${T}_prof_$name.log rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o run -- "$@" || return $?
  local db; db=$(find /tmp/prof_$name -name '*results.db' | head -1)
  python3 scripts/kstats_db.py "$db" 30 --tokens "$tok" > gpurun_out/${T}_kstats_$name.md && rm -rf /tmp/prof_$name
}
run 300 ${T}_ttft.log python bench/ttft_breakdown.py --message 4 --pages 2 &&
run 300 ${T}_ttft8.log python bench/ttft_breakdown.py --message 4 --pages 2 --peers 8 &&
run 600 ${T}_bench.log python bench.py --steps 20 --warmup 5 &&
prof ttft8 300 0 python3 bench/ttft_breakdown.py --message 4 --pages 2 --peers 8 --iters 20 &&
prof ttft 300 0 python3 bench/ttft_breakdown.py --message 4 --pages 2 --iters 20 &&
prof bench 600 0 python3 bench.py --steps 3 --warmup 1 &&
prof proxy 600 0 python3 bench/tp_rank_proxy.py --steps 3 --warmup 1
