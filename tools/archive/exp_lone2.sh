set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 100 python -u tools/lone_path_latency.py cornell34 4=64 > gpurun_out/lone2_c64.jsonl &&
timeout -k 10 100 python -u tools/lone_path_latency.py cornell34 4=64 2=0 14=0 15=0 > gpurun_out/lone2_c64_exits0.jsonl &&
timeout -k 10 100 python -u tools/lone_path_latency.py blob70k 4=64 > gpurun_out/lone2_blob_c64.jsonl &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/drain3 -o run -- python -u tools/drain_export_ab.py --scene cornell34 --strides 8 --passes 1 --steps 3 --settings 0:0,8:1,8:2,8:7,4:2,16:1 > gpurun_out/drain3.jsonl
