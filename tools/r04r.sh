#!/bin/bash
# Round-4 GPU pass r: first hops 8 nodes per thread (ORH_HOP_NODES=8, 104
# VGPRs: one wave fits beside two MS-BFS workgroups) vs 16: sweep parity with
# it, one sweep alone and the 4-lane step each.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04r}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/tests8.log" env ORH_HOP_NODES=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v -k "sweep_all or first_hops_exact or ladder" --timeout 300 --timeout-method thread
for R in 1 2; do
  step "$OUT/sweep16_$R.log" timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step16_$R.log" env T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
  step "$OUT/sweep8_$R.log" env ORH_HOP_NODES=8 timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step8_$R.log" env ORH_HOP_NODES=8 T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
done
echo "r04r done"
