set -o pipefail
timeout -k 10 100 python -u tools/lone_path_latency.py cornell34 > gpurun_out/lone_cornell.jsonl &&
timeout -k 10 100 python -u tools/lone_path_latency.py cornell34 5=1 > gpurun_out/lone_cornell_bpc1.jsonl &&
timeout -k 10 100 python -u tools/lone_path_latency.py cornell34 2=0 > gpurun_out/lone_cornell_wt0.jsonl &&
timeout -k 10 100 python -u tools/lone_path_latency.py blob70k > gpurun_out/lone_blob.jsonl
