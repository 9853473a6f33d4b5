# A/B: the pinned launch table vs an online re-tune on this box (P2P_AUTOTUNE_TABLE=0)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/tb_pin_$i.log 2>&1 || exit 1
  P2P_AUTOTUNE_TABLE=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/tb_live_$i.log 2>&1 || exit 1
done
for f in gpurun_out/tb_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ttft_p50_ms": [0-9.]*' $f)"; done
grep -o '"gemm_autotune": {[^}]*}' gpurun_out/tb_live_1.log
