set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python bench/tp_rank_proxy.py > gpurun_out/r5i_proxy.log 2>&1 || { tail -20 gpurun_out/r5i_proxy.log; exit 1; }
tail -1 gpurun_out/r5i_proxy.log
P2P_DECODE_ENGINE=1 timeout -k 10 500 python bench/tp_rank_proxy.py > gpurun_out/r5i_proxy_de.log 2>&1 || { tail -20 gpurun_out/r5i_proxy_de.log; exit 1; }
tail -1 gpurun_out/r5i_proxy_de.log
