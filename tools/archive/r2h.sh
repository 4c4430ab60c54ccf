set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2h
export TMPDIR=/tmp
timeout -k 10 300 bash tools/ab.sh cornell34 5 nospill ldspad > gpurun_out/r2h/ab_cornell.txt 2>&1 || exit 1
for v in nospill ldspad; do
  export HIPPT_LIB=qt-raytracer_amd/libv_$v.so
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/r2h/pmc_$v -o run -- python3 tools/sweep.py --scene cornell34 --steps 1 > gpurun_out/r2h/pmc_$v.log 2>&1 || exit 1
done
