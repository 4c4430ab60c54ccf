set -o pipefail
export HIPPT_LIB=qt-raytracer_amd/libv_rate.so
timeout -k 10 240 python tools/rate_timeline.py --jobs 1:64,8:64,1:8,8:8 > gpurun_out/rate_e1_default.jsonl &&
timeout -k 10 240 python tools/rate_timeline.py --jobs 1:64,8:64,1:8 28=0 > gpurun_out/rate_e1_noorder.jsonl &&
timeout -k 10 240 python tools/rate_timeline.py --jobs 1:64,8:64,1:8 26=0 > gpurun_out/rate_e1_nopool.jsonl
