set -e
mkdir -p gpurun_out/r06aj
for rep in 1 2; do
  echo "[shipped rep$rep] $(T=32 LANES=2,3 timeout -k 10 300 python tools/lanes_probe.py | tr '\n' ' ')" | tee -a gpurun_out/r06aj/lanes_ab.txt
  echo "[defer low rep$rep] $(ORH_MS_DEFER=1 ORH_MS_DEFER_PRIO=1 T=32 LANES=2,3,4 timeout -k 10 300 python tools/lanes_probe.py | tr '\n' ' ')" | tee -a gpurun_out/r06aj/lanes_ab.txt
done
