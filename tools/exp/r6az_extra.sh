# round 6: the final library's app path (tools/legacy_abi_bench.py: cudaPathTracerRender per frame and
# the present hand-off at 1080p) and kernel-trace profiles of configs[3] (4K/256 spp) and configs[4]
# (the wavefront) -> gpurun_out/r6az/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6az
mkdir -p $O
sha256sum qt-raytracer_amd/libhippt.so > $O/lib.sha256
timeout -k 10 300 python3 -u tools/legacy_abi_bench.py > $O/legacy_abi_1080p.json 2> $O/legacy.err || { tail -20 $O/legacy.err; exit 1; }
cat $O/legacy_abi_1080p.json | head -c 1500; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_4k -o run -- \
  python3 bench.py --preset config4 --steps 3 --warmup 1 --cpu-baseline off > $O/kt_4k_bench.json 2> $O/kt_4k.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_wf -o run -- \
  python3 bench.py --preset config5 --steps 20 --warmup 5 --cpu-baseline off > $O/kt_wf_bench.json 2> $O/kt_wf.err || exit 1
for d in kt_4k kt_wf; do echo $d; head -8 $O/$d/run_kernel_stats.csv; done
echo EXTRA_DONE
