# s7t: tail finish on by default for the camera-pool kernel over global trees: full GPU suite,
# smoke, the headline line, configs[2] and the blob70k 1/8 share
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7t
mkdir -p $O
bash tools/gpu_tests.sh s7t && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err && \
timeout -k 10 300 python -u bench.py --preset config3 --cpu-baseline off > $O/bench_config3.json 2> $O/bench_config3.err && \
timeout -k 10 200 python -u tools/band_scaling.py --scene blob70k --all-bands --ranks 8 > $O/share_blob.jsonl 2>&1
echo "s7t rc=$?"
