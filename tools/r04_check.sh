#!/bin/bash
# Round-4 GPU pass: the new tests first, the whole GPU suite, the C5 leg.
# A pytest exit of 1 (test failures) goes on to the next step; any other
# non-zero exit (crash, abort, time limit) ends the script there.
# usage (repo root, via gpurun): tools/r04_check.sh TAG
TAG=${1:-r04}
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
step "$OUT/new_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_policy.py tests/test_gpu_multi_device.py tests/test_gpu_ksp2_abi.py -v --timeout 300 --timeout-method thread
step "$OUT/gpu_tests.log" timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step "$OUT/bench_c5.json" timeout -k 10 600 python -u bench.py --legs c5,c4 --no-cpu-baseline --steps 5 --warmup 2
echo "r04_check $TAG done"
