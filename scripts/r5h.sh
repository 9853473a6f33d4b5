set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for loop in 1 0; do
  ENGINE_NATIVE_LOOP=$loop timeout -k 10 500 python bench/serve_bench.py --gpus 2 --tp 2 --virtual 1 --kv-pages 2048 --peers 8 --requests 4 > gpurun_out/r5h_serve_tp2_loop$loop.log 2>&1 || { tail -20 gpurun_out/r5h_serve_tp2_loop$loop.log; exit 1; }
  tail -1 gpurun_out/r5h_serve_tp2_loop$loop.log
done
