#!/bin/bash
# Round-4 GPU pass l: what-if slot tier pushed by delta-stepping. What-if
# tests (incl. push vs sweeps, C4 batch vs the oracle), the C4 job timeline
# with and without the push, the C4 leg.
TAG=${1:-r04l}
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
step "$OUT/whatif_tests.log" timeout -k 10 900 python -u -m pytest tests/test_gpu_whatif_repair.py -v --timeout 600 --timeout-method thread
step "$OUT/c4_push.log" timeout -k 10 300 python -u tools/c4_leg.py
step "$OUT/c4_sweeps.log" env ORH_WHATIF_PUSH=0 timeout -k 10 300 python -u tools/c4_leg.py
echo "r04l $TAG done"
