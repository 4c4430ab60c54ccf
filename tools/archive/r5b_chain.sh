# round 5: chained batches — diagnostic sequences, parity subset, then the Cornell / blob70k whole
# image and 1/8 share, chain automatic vs off (option 30 = HIPPT_OPT_CHAIN), 20 steps each
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 200 python -u tools/exp/chain_debug.py cornell34 > gpurun_out/r5b/dbg_cornell.txt 2>&1 || { cat gpurun_out/r5b/dbg_cornell.txt; exit 1; }
cat gpurun_out/r5b/dbg_cornell.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_lifecycle.py -x -v --timeout 200 --timeout-method thread -k "chained or deferred_combine or headline_image or async or lifecycle or exit" > gpurun_out/r5b/pytest.log 2>&1 || { tail -30 gpurun_out/r5b/pytest.log; exit 1; }
tail -3 gpurun_out/r5b/pytest.log
for sc in cornell34 blob70k; do
  for ch in -1 0; do
    timeout -k 10 200 python -u tools/band_scaling.py --scene $sc --steps 20 --ranks 1,8 28=1 30=$ch > gpurun_out/r5b/${sc}_chain${ch}.jsonl || exit 1
  done
done
for f in gpurun_out/r5b/*.jsonl; do echo $f; cat $f; done
