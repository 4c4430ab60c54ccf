# r6r: pair-packed primitive records for triangle-only global trees — GPU suite, then blob70k A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=gpurun_out/r6r
mkdir -p $T
bash tools/gpu_tests.sh r6r && \
timeout -k 10 400 bash tools/ab.sh blob70k 4 pr0 pr1 > $T/ab_pair_records_blob.txt 2>&1 && \
timeout -k 10 400 bash tools/ab.sh blob70k 4 pr1 pr0 >> $T/ab_pair_records_blob.txt 2>&1
echo "r6r rc=$?"
