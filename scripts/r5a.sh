set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py > gpurun_out/r5a_bench.log 2>&1 && tail -1 gpurun_out/r5a_bench.log &&
PROBE_SPLITS=0,1,2,4 timeout -k 10 300 python bench/wide_stamp_probe.py > gpurun_out/r5a_stamp.jsonl 2>&1 && cat gpurun_out/r5a_stamp.jsonl
