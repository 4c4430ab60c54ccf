# r4b: LLVM machine-scheduler strategies (max-ilp, max-memory-clause, AMDGPU register-pressure
# trackers, relaxed occupancy) against the default build, alternating A/B per scene
# (variants: tools/build_variants.sh base="" ilp="-mllvm -amdgpu-sched-strategy=max-ilp"
#  mclause="-mllvm -amdgpu-sched-strategy=max-memory-clause" trk="-mllvm -amdgpu-use-amdgpu-trackers=1"
#  relax="-mllvm -amdgpu-schedule-relaxed-occupancy=1")
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
V="base ilp mclause trk relax"
bash tools/ab.sh cornell34 5 $V > gpurun_out/r4b/ab_cornell.txt 2>&1 && \
bash tools/ab.sh blob70k 4 $V > gpurun_out/r4b/ab_blob.txt 2>&1 && \
bash tools/ab.sh cornell_mixed 4 $V > gpurun_out/r4b/ab_mixed.txt 2>&1 && \
bash tools/ab.sh random_scene 4 $V > gpurun_out/r4b/ab_random.txt 2>&1
python3 tools/ab_summary.py gpurun_out/r4b/ab_*.txt
