set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/drain2 -o run -- python -u tools/drain_export_ab.py --scene cornell34 --strides 8 --passes 1 --steps 3 --settings 0:0,64:2,64:7,16:7 > gpurun_out/drain2.jsonl
