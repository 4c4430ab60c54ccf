set -o pipefail
timeout -k 10 150 python -u tools/drain_export_ab.py --scene cornell34 --strides 8,1 --settings 0:0,16:2,32:2,64:2,32:1,32:4 > gpurun_out/drain1_cornell.jsonl &&
timeout -k 10 200 python -u tools/drain_export_ab.py --scene blob70k --strides 8,1 --steps 3 --settings 0:0,16:2,32:2,64:2,32:4 > gpurun_out/drain1_blob.jsonl
