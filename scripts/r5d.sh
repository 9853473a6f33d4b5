set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PROBE_SPLITS=0 timeout -k 10 300 python bench/wide_stamp_probe.py > gpurun_out/r5d_stamp.jsonl 2>&1 && cat gpurun_out/r5d_stamp.jsonl
