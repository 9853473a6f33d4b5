# Mid-M launch candidates after the granule seam; per-XCD / per-slice stamp arrival.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 300 r5t_stamp.jsonl python bench/wide_stamp_probe.py qkv o_proj down &&
run 500 r5t_pick.jsonl python bench/midm_pick_check.py
