# r3a: re-entry check of HEAD on the box: GPU parity suite, smoke, one default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3a
bash tools/gpu_tests.sh r3a && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3a/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/r3a/cornell.json 2> gpurun_out/r3a/cornell.err && cat gpurun_out/r3a/cornell.json
