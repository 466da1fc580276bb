#!/bin/bash
# Round-4 GPU pass ae: first-hop workgroups per source (ORH_HOP_SPLIT 1 =
# default on C2, 2, 5): one sweep alone, the step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ae}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for S in 1 2 5; do
  step "$OUT/sweep_s$S.log" env ORH_HOP_SPLIT=$S timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step_s$S.log" env ORH_HOP_SPLIT=$S T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
done
echo "r04ae done"
