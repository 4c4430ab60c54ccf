# s7s: tail finish (HIPPT_TAIL_FINISH: drained waves traverse to the end before shading) —
# parity on the variant, then 1/8-share and full-size rates against the default, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s7s
mkdir -p $O
HIPPT_LIB=qt-raytracer_amd/libv_fin1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not wavefront" > $O/pytest_fin1.log 2>&1 && \
for pass in 1 2; do
  for v in fin0 fin1; do
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python -u tools/band_scaling.py --scene cornell34 --all-bands --ranks 1,8 > $O/share_cornell_${v}_p$pass.jsonl 2>&1 || exit 1
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 200 python -u tools/band_scaling.py --scene blob70k --all-bands --ranks 8 > $O/share_blob_${v}_p$pass.jsonl 2>&1 || exit 1
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/sweep.py --scene cornell34 --steps 5 > $O/full_cornell_${v}_p$pass.txt 2>&1 || exit 1
    HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python -u tools/sweep.py --scene blob70k --steps 3 > $O/full_blob_${v}_p$pass.txt 2>&1 || exit 1
  done
done
echo "s7s rc=$?"
