set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/kw_base_$i.log 2>&1 || exit 1
  P2P_QA_WAVES=131072 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/kw_2_$i.log 2>&1 || exit 1
done
for f in gpurun_out/kw_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ttft_p50_ms": [0-9.]*' $f)"; done
