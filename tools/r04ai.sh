#!/bin/bash
# Round-4 GPU pass ai: MS-BFS threads per workgroup (512 default / 768 /
# 1024) with frontier reads in groups of 2: one sweep alone, the step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ai}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for B in 512 768 1024; do
  step "$OUT/sweep_b$B.log" env ORH_MS_BLOCK=$B timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step_b$B.log" env ORH_MS_BLOCK=$B T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
done
echo "r04ai done"
