# round 5: chained batches — kernel time per batch against the cap (1 = structurally the unchained
# fused design), Cornell whole image and 1/8 share; kernel traces and one PMC pass (VALU, LDS, waves)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g
mkdir -p $O
for r in 8 1; do
  for ch in 0 1 2 4 8; do
    timeout -k 10 100 python -u tools/band_scaling.py --scene cornell34 --steps 20 --ranks $r 28=1 30=$ch > $O/cornell_r${r}_chain${ch}.jsonl || exit 1
    echo "r$r chain$ch $(cat $O/cornell_r${r}_chain${ch}.jsonl)"
  done
done
for ch in 0 1 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_r8_c$ch -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 30=$ch > $O/kt_r8_c$ch.jsonl 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -T --output-format csv -d $O/pmc_r8_c$ch -o run -- \
      python3 tools/band_scaling.py --scene cornell34 --steps 20 --ranks 8 28=1 30=$ch > $O/pmc_r8_c$ch.jsonl 2>&1 || exit 1
done
