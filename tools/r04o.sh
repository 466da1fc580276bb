#!/bin/bash
# Round-4 GPU pass o: C2 buildRouteDb phase profile; KSP2 stage times at
# ORH_DELTA_PCT 25 / 50 / 100 / 200 (the u16 LDS searches' bucket width).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04o}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/route_prof.log" timeout -k 10 300 python -u tools/route_prof.py --reps 9
for D in 25 50 100 200; do
  step "$OUT/ksp_delta$D.log" env ORH_DELTA_PCT=$D timeout -k 10 200 python -u tools/ksp2_stage_ab.py 1
done
echo "r04o done"
