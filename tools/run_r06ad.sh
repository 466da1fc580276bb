set -e
bash tools/gpu_round.sh r06ad
timeout -k 10 300 python tools/c4_multi_device_rehearsal.py 2 4 8 > gpurun_out/r06ad/rehearsal.jsonl 2>&1
