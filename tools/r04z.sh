#!/bin/bash
# Round-4 GPU pass z: nexthop-set cache A/B on one box (ORH_NH_CACHE=1 / 0,
# alternating): C2 route profile and the C3 / C5 legs.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04z}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for R in 1 2; do
  for C in 1 0; do
    step "$OUT/route_prof_c${C}_$R.log" env ORH_NH_CACHE=$C ORH_MALLOC_TUNE=1 timeout -k 10 200 python -u tools/route_prof.py --reps 9
    step "$OUT/legs_c${C}_$R.json" env ORH_NH_CACHE=$C timeout -k 10 300 python -u bench.py --legs c3,c5 --no-cpu-baseline --steps 2 --warmup 1
  done
done
echo "r04z done"
