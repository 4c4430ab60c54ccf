# r2t: top of the tree in LDS (HIPPT_OPT_LDS_TOP_NODES) x LDS stack cap, global-memory trees
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2t
timeout -k 10 100 python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread -k "quant or spill or wide or random or blob" > gpurun_out/r2t/pytest.log 2>&1 && \
timeout -k 10 300 python tools/sweep.py --scene blob70k --steps 3 --count stackcap=19,17,15,13 top=0,5,21,85,-1 > gpurun_out/r2t/blob.jsonl && \
timeout -k 10 200 python tools/sweep.py --scene random_scene --steps 3 top=0,-1 > gpurun_out/r2t/random.jsonl && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 stackcap=19 top=0,-1 top=0,-1 > gpurun_out/r2t/blob_repeat.jsonl
