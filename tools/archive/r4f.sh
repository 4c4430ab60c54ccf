# r4f: wave priority raised while a 4-wide node's rows are loaded (HIPPT_SETPRIO 1 / 3) vs the
# default build, alternating A/B
# (the HIPPT_SETPRIO experiment code was removed from hippt_trace.h after this measurement)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4f
V="base prio1 prio3"
bash tools/ab.sh blob70k 4 $V > gpurun_out/r4f/ab_blob.txt 2>&1 && \
bash tools/ab.sh cornell34 5 $V > gpurun_out/r4f/ab_cornell.txt 2>&1 && \
bash tools/ab.sh random_scene 4 $V > gpurun_out/r4f/ab_random.txt 2>&1 && \
bash tools/ab.sh cornell_mixed 4 $V > gpurun_out/r4f/ab_mixed.txt 2>&1
python3 tools/ab_summary.py gpurun_out/r4f/ab_*.txt
