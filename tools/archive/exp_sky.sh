set -o pipefail
for i in 1 2; do
timeout -k 10 100 python -u tools/drain_export_ab.py --scene cornell34 --strides 8 --passes 2 --settings 0:0,16:7,32:7 > gpurun_out/sky_new_$i.jsonl &&
HIPPT_LIB=qt-raytracer_amd/libv_oldsky.so timeout -k 10 100 python -u tools/drain_export_ab.py --scene cornell34 --strides 8 --passes 2 --settings 0:0,16:7,32:7 > gpurun_out/sky_old_$i.jsonl || exit 1
done
HIPPT_LIB=qt-raytracer_amd/libv_rate.so timeout -k 10 100 python -u tools/rate_timeline.py --jobs 8:64,1:8 > gpurun_out/rate_sky.jsonl
