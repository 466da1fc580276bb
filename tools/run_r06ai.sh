set -e
mkdir -p gpurun_out/r06ai
for rep in 1 2; do
  for V in "" "ORH_MS_DEFER=1 ORH_MS_DEFER_PRIO=1" "ORH_MS_DEFER=1 ORH_MS_DEFER_PRIO=-1"; do
    echo "[${V:-shipped} rep$rep] $(env $V T=32 LANES=2 timeout -k 10 200 python tools/lanes_probe.py)" | tee -a gpurun_out/r06ai/prio_ab.txt
  done
done
