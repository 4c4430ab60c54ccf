# round 6: the final kernels' loop exits, wave threshold, chunk and LDS top re-swept in one process per
# scene (tools/sweep.py, 200 ms warm-up, 5 timed steps per setting, two passes) -> gpurun_out/r6ad/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ad
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 leafexit=12,17,24,32 nodeexit=32,48,64 > $O/blob_exits_p$pass.jsonl 2> $O/blob_exits_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene cornell34 --steps 10 leafexit=8,12,16 nodeexit=4,8,12,16 > $O/cornell_exits_p$pass.jsonl 2> $O/cornell_exits_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 wave=-1,16,24,32,40 chunk=256,512,1024 > $O/blob_wave_p$pass.jsonl 2> $O/blob_wave_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene cornell34 --steps 10 wave=-1,16,24,32,40 chunk=256,512,1024 > $O/cornell_wave_p$pass.jsonl 2> $O/cornell_wave_p$pass.err || exit 1
done
echo SWEEP_DONE
