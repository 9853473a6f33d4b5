# kernel table of the 8-peer prompt chunk (which gate_up tile runs)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof8 -o run -- python3 bench/ttft_breakdown.py --message 4 --pages 2 --peers 8 --iters 20 > gpurun_out/r5h4_prof.log 2>&1 || exit $?
db=$(find /tmp/prof8 -name '*results.db' | head -1)
python3 scripts/kstats_db.py "$db" 16 > gpurun_out/r5h4_kstats.md && cat gpurun_out/r5h4_kstats.md
