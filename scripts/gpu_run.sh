#!/bin/bash
# One parametrized GPU session script (replaces the per-experiment r3_gpu_*.sh wrappers).
# Usage: STEPS="ttft,bench,tests,smoke,prof,pmc,serve,proxy,cmd" [env knobs] bash scripts/gpu_run.sh
# Every GPU step runs under its own time limit; the first failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench}
TAG=${TAG:-run}
step() {  # step <name> <timeout> <log> cmd...
  local name=$1 lim=$2 log=$3; shift 3
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
IFS=',' read -ra S <<< "$STEPS"
for s in "${S[@]}"; do
  case "$s" in
    tests) step tests ${TEST_TIMEOUT:-900} "${TAG}_pytest_gpu.log" python -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -q \
             --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke) step smoke 300 "${TAG}_smoke.log" python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 "${TAG}_bench.log" python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} ;;
    bench8) step bench8 600 "${TAG}_bench_p8.log" python bench.py --peers 8 --steps 10 --warmup 3 ;;
    ttft) step ttft 300 "${TAG}_ttft.log" python bench/ttft_breakdown.py ${TTFT_ARGS:-} ;;
    prof) step prof 600 "${TAG}_prof.log" rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run \
             -- python3 bench.py --steps 3 --warmup 1 ;;
    serve) step serve 600 "${TAG}_serve.log" python bench/serve_bench.py ${SERVE_ARGS:-} ;;
    proxy) step proxy 600 "${TAG}_proxy.log" python bench/tp_rank_proxy.py ${PROXY_ARGS:-} ;;
    pmc)  # PMC passes over PMC_CMD (a python3 command line), one counter set per run.  Keep
          # the target short: counter collection serialises every kernel, and a run silent for
          # 3 minutes is killed (the whole headline bench with its start-up autotune is too long)
      [ -n "${PMC_CMD:-}" ] || { echo "pmc: set PMC_CMD"; exit 2; }
      i=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
                 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS" \
                 "FETCH_SIZE TCP_TCC_READ_REQ_sum"; do
        i=$((i+1))
        step pmc$i 300 "${TAG}_pmc$i.log" rocprofv3 --pmc $set --kernel-trace -d gpurun_out/${TAG}_pmc$i -o run \
             -- python3 $PMC_CMD
      done ;;
    cmd) step cmd ${CMD_TIMEOUT:-600} "${TAG}_cmd.log" bash -c "$CMD" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps ok"
