#!/bin/bash
# Round-4 GPU pass ad: KSP2 u16 LDS search threads per search (1024 default,
# 768, 512) and bucket width around 50 %.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ad}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for B in 1024 768 512; do
  step "$OUT/ksp_b$B.log" env ORH_LDS16_BLOCK=$B timeout -k 10 200 python -u tools/ksp2_stage_ab.py 1
done
for D in 35 70; do
  step "$OUT/ksp_d$D.log" env ORH_DELTA_PCT=$D timeout -k 10 200 python -u tools/ksp2_stage_ab.py 1
done
echo "r04ad done"
