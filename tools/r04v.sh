#!/bin/bash
# Round-4 GPU pass v: MS-BFS frontier-read group size (2 / 4 = default / 5 /
# 10 owned nodes per batch of LDS reads): one sweep alone, the 4-lane step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04v}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for V in base g2 g5 g10; do
  if [ $V = base ]; then L=$ROOT/openr_amd/lib; else L=$ROOT/build_var/$V; fi
  step "$OUT/sweep_$V.log" env LD_LIBRARY_PATH=$L timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step_$V.log" env LD_LIBRARY_PATH=$L T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
done
echo "r04v done"
# latency plan (1,024 threads when every batch has a CU) vs 512 threads for a shard
step "$OUT/strong_lat1.log" timeout -k 10 300 python -u tools/strong_rehearsal.py 100 1 2 4 8
step "$OUT/strong_lat0.log" env ORH_MS_LATENCY=0 timeout -k 10 300 python -u tools/strong_rehearsal.py 100 1 2 4 8
echo "r04v strong done"
