set -e
mkdir -p gpurun_out/r06ab
for V in "" ORH_WHATIF_SEARCH_CAP=8 ORH_WHATIF_SEARCH_CAP=32; do
  env $V timeout -k 10 300 python tools/c4_multi_device_rehearsal.py 4 8 > gpurun_out/r06ab/rehearsal_${V:-shipped}.jsonl 2>&1
done
