# round 4: chained batches (HIPPT_OPT_CHAIN): parity first, then the 1/8 share and the whole image
# with one launch per batch (30=0), chained (30=1) and automatic (30=-1), alternating
set -o pipefail
mkdir -p gpurun_out/r4r
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chained or deferred_combine or item_order or camera_pool or fuse" > gpurun_out/r4r/pytest_chain.log 2>&1 || exit 1
for i in 1 2; do
  for ch in 0 1 -1; do
    for scene in cornell34 blob70k; do
      timeout -k 10 150 python -u tools/band_scaling.py --scene $scene --steps 10 --ranks 1,8 28=1 30=$ch > gpurun_out/r4r/${scene}_chain${ch}_$i.jsonl || exit 1
    done
  done
done
