#!/bin/bash
# Round-4 GPU pass ag: oversized slot-tier repairs searched in full
# (ORH_WHATIF_BIG): what-if tests, then the C4 leg with and without.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ag}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/whatif_tests.log" timeout -k 10 700 python -u -m pytest tests/test_gpu_whatif_repair.py -v --timeout 600 --timeout-method thread
step "$OUT/c4_big.log" timeout -k 10 300 python -u tools/c4_leg.py
step "$OUT/c4_nobig.log" env ORH_WHATIF_BIG=0 timeout -k 10 300 python -u tools/c4_leg.py
step "$OUT/c4_big4k.log" env ORH_WHATIF_BIG=4096 timeout -k 10 300 python -u tools/c4_leg.py
echo "r04ag done"
