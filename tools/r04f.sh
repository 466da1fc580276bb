#!/bin/bash
# Round-4 GPU pass f: the u16-LDS KSP2 tests (spill table), the KSP2 stage
# timing, then the PMC profile of the C2 sweep kernels alone (one topology,
# one lane: what roofline.traffic describes) and of the 4-lane step.
TAG=${1:-r04f}
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
step "$OUT/ksp_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_ksp2_abi.py -v -k "lds16" --timeout 300 --timeout-method thread
step "$OUT/latency_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v -k "latency_plan" --timeout 300 --timeout-method thread --timeout 300 --timeout-method thread
step "$OUT/strong.log" timeout -k 10 300 python -u tools/strong_rehearsal.py 100 1 2 4 8
step "$OUT/ksp_stage.log" timeout -k 10 300 python -u tools/ksp2_stage_ab.py 1
step "$OUT/prof_one.log" timeout -k 10 900 bash tools/profile.sh ${TAG}_one --topologies 1 --lanes 1 --steps 10 --warmup 2 --no-cpu-baseline --no-route-db --legs=
step "$OUT/prof_step.log" timeout -k 10 900 bash tools/profile.sh ${TAG}_step --steps 5 --warmup 2 --no-cpu-baseline --no-route-db --legs=
echo "r04f $TAG done"
