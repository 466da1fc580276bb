#!/bin/bash
# Round-4 GPU pass m: the whole GPU suite and smoke on the final kernels, then
# the kernel trace + PMC passes of the isolated C2 sweep (roofline.traffic).
TAG=${1:-r04m}
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
step "$OUT/gpu_tests.log" timeout -k 10 780 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step "$OUT/smoke.log" timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step "$OUT/prof_one.log" timeout -k 10 400 bash tools/profile.sh ${TAG}_one --topologies 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline --no-route-db --legs=
echo "r04m $TAG done"
