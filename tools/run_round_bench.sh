set -e
mkdir -p gpurun_out/r1d
B="timeout -k 10 300 python3 bench.py"
$B > gpurun_out/r1d/cornell.json 2> gpurun_out/r1d/cornell.err
$B --scene blob70k --cpu-baseline off > gpurun_out/r1d/blob.json 2>> gpurun_out/r1d/err
$B --scene blob70k --width 3840 --height 2160 --spp 256 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r1d/blob4k.json 2>> gpurun_out/r1d/err
$B --scene blob70k --path-mode wavefront --cpu-baseline off > gpurun_out/r1d/blob_wf.json 2>> gpurun_out/r1d/err
$B --scene random_scene --cpu-baseline off > gpurun_out/r1d/random.json 2>> gpurun_out/r1d/err
$B --scene cornell_mixed --cpu-baseline off > gpurun_out/r1d/mixed.json 2>> gpurun_out/r1d/err
bash tools/profile.sh r1d
bash tools/profile.sh r1d_blob --scene blob70k
echo ALLDONE
