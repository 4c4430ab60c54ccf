# s7m: wavefront extend over half-precision planes: parity, then configs[4] (blob70k wavefront)
# with 8-bit (default), half and float nodes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7m
mkdir -p $O
bash tools/gpu_tests.sh s7m "wavefront" && \
for pass in 1 2; do
  for q in -1 3 0; do
    timeout -k 10 200 python -u bench.py --preset config5 --steps 5 --warmup 1 --cpu-baseline off --option BVH_QUANT=$q > $O/wf_quant${q}_p$pass.json 2> $O/wf_quant${q}_p$pass.err || exit 1
  done
done
echo "s7m rc=$?"
