#!/bin/bash
# Round-4 GPU pass g: MS-BFS arrival log. Sweep parity (C2 all sources,
# drained variants, latency plan, u16 masks, deep levels, Clos), the KSP2
# spill test, then the step / sweep timing with the log and without it
# (ORH_MS_LOG=0), and a PMC pass of the isolated sweep.
TAG=${1:-r04g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/sweep_tests.log" timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multi_device.py -v -k "sweep or latency or ladder or u16 or clos or c3 or multi_device" --timeout 300 --timeout-method thread
step "$OUT/ksp_tests.log" timeout -k 10 300 python -u -m pytest tests/test_gpu_ksp2_abi.py -v -k "spill" --timeout 200 --timeout-method thread
for L in 1 0; do
  step "$OUT/step_log$L.log" env ORH_MS_LOG=$L T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
  step "$OUT/sweep_log$L.log" env ORH_MS_LOG=$L timeout -k 10 120 python -u tools/quick_bench.py
done
step "$OUT/prof_one.log" timeout -k 10 900 bash tools/profile.sh ${TAG}_one --topologies 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline --no-route-db --legs=
echo "r04g $TAG done"
