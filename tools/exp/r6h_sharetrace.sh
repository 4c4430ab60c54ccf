# round 6: kernel trace of the 1/8 row share's 20-step burst (Cornell and blob70k, rank 0): every
# launch's duration and gap -> gpurun_out/r6h/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6h
mkdir -p $O
for sc in cornell34 blob70k; do
  timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $O/kt_$sc -o run -- \
    python3 tools/band_scaling.py --scene $sc --steps 20 --ranks 8 28=1 > $O/share8_$sc.jsonl 2> $O/share8_$sc.err || exit 1
done
echo TRACE_DONE
