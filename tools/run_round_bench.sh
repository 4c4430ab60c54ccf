# tools/run_round_bench.sh TAG — run ON THE GPU BOX (via gpurun): the bench lines of every
# BASELINE config plus the rocprof profiles of the two headline scenes, into gpurun_out/TAG/.
set -e
TAG=${1:?tag}
mkdir -p gpurun_out/$TAG
B="timeout -k 10 300 python3 bench.py"
bash tools/profile.sh $TAG
bash tools/profile.sh ${TAG}_blob --scene blob70k
python3 tools/prof_summary.py $TAG > /dev/null
python3 tools/prof_summary.py ${TAG}_blob > /dev/null
$B > gpurun_out/$TAG/cornell.json 2> gpurun_out/$TAG/cornell.err
$B --scene blob70k > gpurun_out/$TAG/blob.json 2>> gpurun_out/$TAG/err
$B --scene blob70k --width 3840 --height 2160 --spp 256 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/$TAG/blob4k.json 2>> gpurun_out/$TAG/err
$B --scene blob70k --path-mode wavefront --cpu-baseline off > gpurun_out/$TAG/blob_wf.json 2>> gpurun_out/$TAG/err
$B --scene random_scene --cpu-baseline off > gpurun_out/$TAG/random.json 2>> gpurun_out/$TAG/err
$B --scene cornell_mixed --cpu-baseline off > gpurun_out/$TAG/mixed.json 2>> gpurun_out/$TAG/err
echo ALLDONE
