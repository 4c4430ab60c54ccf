# r2za: wavefront extend with the LDS top of the tree: float vs 8-bit nodes (blob70k)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2za
timeout -k 10 100 python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread -k "wavefront or top" > gpurun_out/r2za/pytest.log 2>&1 && \
timeout -k 10 400 python tools/sweep.py --scene blob70k --steps 2 mode=1 quant=1,0 top=0,-1 > gpurun_out/r2za/blob_wf.jsonl
