# round 6: the new big-batch defaults on blob70k (whole image, 4K) against the previous ones through
# --option, and the wavefront's extend thresholds (wave / leaf / node exits) -> gpurun_out/r6aq/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6aq
mkdir -p $O
for pass in 1 2; do
  for e in new old; do
    A=""; [ $e = old ] && A="--wave-threshold 40 --option LEAF_EXIT=17 --option NODE_EXIT=48"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off $A > $O/blob_${e}_p$pass.json 2> $O/blob_${e}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_${e}_p$pass.json'));print('blob70k $e pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
  done
done
for e in new old; do
  A=""; [ $e = old ] && A="--wave-threshold 40 --option LEAF_EXIT=17 --option NODE_EXIT=48"
  timeout -k 10 300 python3 bench.py --preset config4 --steps 5 --warmup 1 --cpu-baseline off $A > $O/blob4k_$e.json 2> $O/blob4k_$e.err || exit 1
  python3 -c "import json;d=json.load(open('$O/blob4k_$e.json'));print('blob4k $e', d['value'], d['ms_per_step'])"
done
for pass in 1 2; do
  for e in 32_17_48 40_22_56 32_22_56 40_17_48 24_17_48; do
    IFS=_ read w l n <<< "$e"
    timeout -k 10 200 python3 bench.py --preset config5 --steps 20 --warmup 5 --cpu-baseline off --wave-threshold $w --option LEAF_EXIT=$l --option NODE_EXIT=$n > $O/wf_${e}_p$pass.json 2> $O/wf_${e}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/wf_${e}_p$pass.json'));print('wavefront $e pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
  done
done
echo WF_DONE
