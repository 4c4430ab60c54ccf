set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 &&
timeout -k 10 120 python tools/phase_profile.py --scene cornell34 > gpurun_out/r2a/phase_cornell.json 2>&1 &&
timeout -k 10 120 python tools/phase_profile.py --scene blob70k > gpurun_out/r2a/phase_blob.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r2a/bench_cornell.json 2>gpurun_out/r2a/bench_cornell.err &&
timeout -k 10 200 python bench.py --scene blob70k --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r2a/bench_blob.json 2>gpurun_out/r2a/bench_blob.err
echo rc=$?
