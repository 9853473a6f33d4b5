# Batched-prompt GEMMs with COLD weights (as inside the model) vs hipBLASLt, incl. the tall SwiGLU form.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 800 python bench/prefill_gemm_bench.py --cold --M 160 288 384 512 --only v2_auto v2_256x256_phased v2_320x128 v2_128x128_s2 v2_192x128 > gpurun_out/r5h5_cold.jsonl 2>&1; rc=$?; tail -2 gpurun_out/r5h5_cold.jsonl; exit $rc
