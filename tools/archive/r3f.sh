# r3f: one prepare/begin site for new rays + a shared 1/sqrt for sky and Lambertian lanes: parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3f
bash tools/gpu_tests.sh r3f && \
timeout -k 10 300 bash tools/ab.sh cornell34 5 pool fresh > gpurun_out/r3f/ab_cornell.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh blob70k 3 pool fresh > gpurun_out/r3f/ab_blob.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh cornell_mixed 3 pool fresh > gpurun_out/r3f/ab_mixed.txt 2>&1 && \
timeout -k 10 300 bash tools/ab.sh random_scene 3 pool fresh > gpurun_out/r3f/ab_random.txt 2>&1 && \
timeout -k 10 120 python tools/phase_profile.py --scene blob70k > gpurun_out/r3f/phase_blob.json 2>&1
