# r2zd: memoized random_in_unit_sphere (16 GiB table) vs the rejection loop
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2zd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rng_table or rng or top" > gpurun_out/r2zd/pytest.log 2>&1 && \
timeout -k 10 200 python tools/sweep.py --scene cornell34 --steps 5 rngtab=0,1 rngtab=0,1 > gpurun_out/r2zd/cornell.jsonl && \
timeout -k 10 200 python tools/sweep.py --scene blob70k --steps 3 rngtab=0,1 > gpurun_out/r2zd/blob.jsonl && \
timeout -k 10 200 python tools/sweep.py --scene random_scene --steps 3 rngtab=0,1 > gpurun_out/r2zd/random.jsonl && \
timeout -k 10 200 python tools/sweep.py --scene cornell_mixed --steps 3 rngtab=0,1 > gpurun_out/r2zd/mixed.jsonl
