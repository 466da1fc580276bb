#!/bin/bash
# Round-4 GPU pass w: link ids loaded with the edge records (searches with
# ignore sets): KSP2 + what-if tests, KSP2 stage times; then pass v's A/Bs.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04w}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/tests.log" timeout -k 10 700 python -u -m pytest tests/test_gpu_ksp2_abi.py tests/test_gpu_whatif_repair.py -q --timeout 300 --timeout-method thread
step "$OUT/ksp_stage.log" timeout -k 10 200 python -u tools/ksp2_stage_ab.py 1
bash tools/r04v.sh r04v
echo "r04w done"
