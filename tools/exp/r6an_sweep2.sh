# round 6: blob70k's loop exits, claim size and stack cap around the defaults with the new wave
# threshold 40 (tools/sweep.py, 200 ms warm-up, 5 timed steps per setting, two passes) -> gpurun_out/r6an/
set -o pipefail
cd /tmp
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6an
mkdir -p $O
for pass in 1 2; do
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 wave=40 leafexit=14,17,20 nodeexit=40,48,56 > $O/blob_exits_p$pass.jsonl 2> $O/blob_exits_p$pass.err || exit 1
  timeout -k 10 300 python3 -u tools/sweep.py --scene blob70k --steps 5 wave=40 chunk=256,512,1024 stackcap=0,8,12 > $O/blob_chunk_p$pass.jsonl 2> $O/blob_chunk_p$pass.err || exit 1
done
echo SWEEP2_DONE
