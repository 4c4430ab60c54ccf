# round 6: blob70k's leaf / node exits with the wave threshold 40 (r6an's sweep: leaf exit 20 +0.8%):
# bench.py A/B, three alternating passes, whole image and the 4K config -> gpurun_out/r6ao/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ao
mkdir -p $O
for pass in 1 2 3; do
  for e in default 20_48 20_56 22_56 24_56; do
    A=""; [ $e != default ] && A="--option LEAF_EXIT=${e%_*} --option NODE_EXIT=${e#*_}"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off $A > $O/blob_e${e}_p$pass.json 2> $O/blob_e${e}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_e${e}_p$pass.json'));print('blob70k exits $e pass $pass', d['value'], d['ms_per_step'], d['config'].get('image_crc32'))"
  done
done
echo EXITS_DONE
