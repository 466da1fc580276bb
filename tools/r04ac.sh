#!/bin/bash
# Round-4 GPU pass ac: MS-BFS group 1 vs 2 (default), first-hop neighbour rows
# in flight 2 / 4 (default) / 8 with 8-node first hops: one sweep, the step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ac}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for V in base g1 hop2 hop8 base2; do
  if [ ${V#base} != $V ]; then L=$ROOT/openr_amd/lib; else L=$ROOT/build_var/$V; fi
  step "$OUT/sweep_$V.log" env LD_LIBRARY_PATH=$L timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step_$V.log" env LD_LIBRARY_PATH=$L T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
done
echo "r04ac done"
