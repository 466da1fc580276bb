#!/bin/bash
# Round-4 GPU pass e: KSP2 LDS-search tests, KSP2 stage A/B, the step A/B of
# library variants, the strong-scaling rehearsal. Stops at the first step
# that crashes, aborts or times out (rc not 0/1).
TAG=${1:-r04e}
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
step "$OUT/ksp_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_ksp2_abi.py -v --timeout 300 --timeout-method thread
step "$OUT/ksp_stage_ab.log" timeout -k 10 300 python -u tools/ksp2_stage_ab.py 1 0
step "$OUT/variant_ab.log" timeout -k 10 900 bash tools/variant_step_ab.sh base msbfs_only nolvl hop1 hop8
step "$OUT/strong.log" timeout -k 10 300 python -u tools/strong_rehearsal.py 100 1 2 4 8
echo "r04e $TAG done"
