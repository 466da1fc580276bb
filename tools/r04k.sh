#!/bin/bash
# Round-4 GPU pass k: KSP2 searches stopped at their targets (all KSP2 tests,
# stage timing with and without ORH_KSP_STOP), then the C4 leg.
TAG=${1:-r04k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/ksp_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_ksp2_abi.py tests/test_ka_decision_more.py -v -m gpu --timeout 300 --timeout-method thread
step "$OUT/ksp_stage_stop.log" timeout -k 10 300 python -u tools/ksp2_stage_ab.py 1
step "$OUT/ksp_stage_nostop.log" env ORH_KSP_STOP=0 timeout -k 10 300 python -u tools/ksp2_stage_ab.py 1
step "$OUT/bench_c4.json" timeout -k 10 600 python -u bench.py --legs c4 --no-cpu-baseline --steps 5 --warmup 2
echo "r04k $TAG done"
