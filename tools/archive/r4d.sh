# r4d: capped unit-sphere draw per shading pass (HIPPT_REJECT_CAP, Lambertian-triangle kernels):
# GPU parity suite on the cap 1 and 2 builds, alternating A/B of caps 1-4, bench CRCs of cap 2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
T="timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
HIPPT_LIB=qt-raytracer_amd/libv_cap2.so $T > gpurun_out/r4d/pytest_cap2.log 2>&1 && tail -1 gpurun_out/r4d/pytest_cap2.log && \
HIPPT_LIB=qt-raytracer_amd/libv_cap1.so $T > gpurun_out/r4d/pytest_cap1.log 2>&1 && tail -1 gpurun_out/r4d/pytest_cap1.log && \
bash tools/ab.sh cornell34 5 base cap1 cap2 cap3 cap4 > gpurun_out/r4d/ab_cornell.txt 2>&1 && \
bash tools/ab.sh blob70k 4 base cap1 cap2 cap3 cap4 > gpurun_out/r4d/ab_blob.txt 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_cap2.so timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/r4d/cornell_cap2.json 2>&1 && \
HIPPT_LIB=qt-raytracer_amd/libv_cap2.so timeout -k 10 300 python3 bench.py --scene blob70k --cpu-baseline off > gpurun_out/r4d/blob_cap2.json 2>&1
python3 tools/ab_summary.py gpurun_out/r4d/ab_*.txt
