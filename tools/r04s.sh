#!/bin/bash
# Round-4 GPU pass s: whole GPU suite + smoke with 8-node first hops, then
# one sweep alone and the step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04s}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/gpu_tests.log" timeout -k 10 780 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step "$OUT/smoke.log" timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step "$OUT/sweep.log" timeout -k 10 120 python -u tools/quick_bench.py
step "$OUT/step.log" env T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
echo "r04s done"
