# round 6: the chain cap of a whole image at the final library (automatic: blob70k 3, Cornell 0 =
# unchained): bench.py A/B, two alternating passes -> gpurun_out/r6aw/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6aw
mkdir -p $O
for pass in 1 2; do
  for c in auto 0 2 6 16; do
    A=""; [ $c != auto ] && A="--option CHAIN=$c"
    timeout -k 10 200 python3 bench.py --scene blob70k --steps 20 --warmup 5 --cpu-baseline off $A > $O/blob_c${c}_p$pass.json 2> $O/blob_c${c}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/blob_c${c}_p$pass.json'));print('blob70k chain $c pass $pass', d['value'], d['ms_per_step'], d['config']['chain']['applied_cap'])"
  done
  for c in auto 2 3 8; do
    A=""; [ $c != auto ] && A="--option CHAIN=$c"
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off $A > $O/cornell_c${c}_p$pass.json 2> $O/cornell_c${c}_p$pass.err || exit 1
    python3 -c "import json;d=json.load(open('$O/cornell_c${c}_p$pass.json'));print('cornell chain $c pass $pass', d['value'], d['ms_per_step'], d['config']['chain']['applied_cap'])"
  done
done
echo CAP_DONE
