#!/bin/bash
# Round-4 GPU pass q: per-slice arrival logs with lane-held counts and
# per-wave assembly: sweep parity, one sweep alone, the 4-lane step, stamps.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04q}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/sweep_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multi_device.py -v -k "sweep or latency or u16 or ladder or clos or multi_device" --timeout 300 --timeout-method thread
step "$OUT/sweep.log" timeout -k 10 120 python -u tools/quick_bench.py
step "$OUT/step.log" env T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
step "$OUT/diag.log" env LD_LIBRARY_PATH=$ROOT/build_var/diag timeout -k 10 120 python -u tools/quick_bench.py
echo "r04q done"
