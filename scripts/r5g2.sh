# Round-5 validation: the world-8 virtual-rank test on its own, then the rest of the GPU tier
# (everything after it alphabetically), smoke and the headline bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 "gpurun_out/$log"; return $rc; }
run 400 r5g2_world8.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_world8_gpu.py -m gpu &&
run 400 r5g2_rest.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_world8_gpu.py -k "not world8" &&
run 300 r5g2_smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
run 600 r5g2_bench.log python bench.py --steps 20 --warmup 5
