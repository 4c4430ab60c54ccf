# r2r: GPU parity suite, per-phase SIMD efficiency (Cornell, blob70k), baseline timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2r
bash tools/gpu_tests.sh r2r && \
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r2r/phase_cornell.json && \
timeout -k 10 120 python tools/phase_profile.py --scene blob70k > gpurun_out/r2r/phase_blob.json && \
timeout -k 10 120 python tools/sweep.py --scene cornell34 --steps 5 > gpurun_out/r2r/base_cornell.jsonl && \
timeout -k 10 120 python tools/sweep.py --scene blob70k --steps 5 > gpurun_out/r2r/base_blob.jsonl
