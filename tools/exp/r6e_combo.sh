# round 6: tile-run parity tests, then the validation lines (r6c) and the tile A/B (r6d)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "tiles" > gpurun_out/r6e/pytest.log 2>&1 || { tail -30 gpurun_out/r6e/pytest.log; exit 1; }
tail -2 gpurun_out/r6e/pytest.log
bash tools/exp/r6c_validate.sh && bash tools/exp/r6d_tiles.sh
