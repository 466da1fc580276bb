set -e
mkdir -p gpurun_out/r06r
for V in "" ORH_WHATIF_FULL=16 ORH_WHATIF_FULL=64; do
  env $V timeout -k 10 300 python tools/c4_multi_device_rehearsal.py 4 8 > gpurun_out/r06r/rehearsal_${V:-shipped}.jsonl 2>&1
done
