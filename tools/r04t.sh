#!/bin/bash
# Round-4 GPU pass t: route-build tests after the fused merge / label pass,
# the C2 route-build profile, the PMC + kernel trace of one C2 sweep (8-node
# first hops).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04t}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/route_tests.log" timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wire.py tests/test_gpu_ingest.py tests/test_ka_decision.py tests/test_ka_decision_more.py tests/test_gpu_policy.py -m gpu -q --timeout 300 --timeout-method thread
step "$OUT/route_prof.log" env ORH_MALLOC_TUNE=1 timeout -k 10 300 python -u tools/route_prof.py --reps 9
step "$OUT/prof_one.log" timeout -k 10 400 bash tools/profile.sh ${1:-r04t}_one --topologies 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline --no-route-db --legs=
echo "r04t done"
