# r3c: camera-ray pool: parity tests, A/B vs the previous commit (rsq), pool on/off sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "camera_pool or mesh_matches or general_scene" > gpurun_out/r3c/pytest.log 2>&1 && \
timeout -k 10 300 bash tools/ab.sh cornell34 5 rsq pool > gpurun_out/r3c/ab_cornell.txt 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell_mixed --steps 3 pool=0,1 pool=0,1 > gpurun_out/r3c/mixed.jsonl 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene random_scene --steps 3 pool=0,1 pool=0,1 > gpurun_out/r3c/random.jsonl 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 pool=0,1 pool=0,1 > gpurun_out/r3c/blob.jsonl 2>&1 && \
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r3c/phase_cornell.json 2>&1
