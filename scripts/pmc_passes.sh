#!/bin/bash
# rocprofv3 --pmc passes over one short python3 target, one counter set per run (the per-block
# slot limits kept: <= 8 SQ, 4 TCC, 4 TCP, 2 GRBM per pass).
# Usage: bash scripts/pmc_passes.sh <out-dir-under-gpurun_out> <python3 args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p "$out"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$out/p$i" -o run -- python3 "$@" > "$out/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/p$i.log"; exit $rc; }
done
find "$out" -name "*counter_collection*"
