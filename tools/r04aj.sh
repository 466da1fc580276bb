#!/bin/bash
# Round-4 GPU pass aj: what-if copy with its loads batched ahead of the
# stores (ORH_WHATIF_COPY=1) vs one load/store pair at a time (default):
# what-if tests, the C4 leg both ways, kernel stats of the copy both ways.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04aj}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/whatif_tests.log" env ORH_WHATIF_COPY=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_whatif_repair.py -v --timeout 600 --timeout-method thread
step "$OUT/c4_batched.log" env ORH_WHATIF_COPY=1 timeout -k 10 300 python -u tools/c4_leg.py
step "$OUT/c4_pairwise.log" timeout -k 10 300 python -u tools/c4_leg.py
step "$OUT/c4_batched2.log" env ORH_WHATIF_COPY=1 timeout -k 10 300 python -u tools/c4_leg.py
cd /tmp && export TMPDIR=/tmp
export ORH_WHATIF_COPY=1
step "$OUT/prof_batched.log" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_batched" -o run -- python3 "$ROOT/tools/c4_leg.py"
unset ORH_WHATIF_COPY
step "$OUT/prof_pairwise.log" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_pairwise" -o run -- python3 "$ROOT/tools/c4_leg.py"
echo "r04aj done"
