#!/bin/bash
# Round-4 GPU pass x: nexthop sets copied from a per-selection cache: route
# build + wire-order tests, the C2 route profile, the C3 / C5 legs; then the
# link-id / KSP2 and MS-BFS A/B passes (w, v).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04x}
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/route_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_policy.py tests/test_gpu_configs.py tests/test_gpu_ingest.py -q -m gpu -k "not sweep_all and not latency" --timeout 300 --timeout-method thread
step "$OUT/route_prof.log" env ORH_MALLOC_TUNE=1 timeout -k 10 200 python -u tools/route_prof.py --reps 9
step "$OUT/bench_c3c5.json" timeout -k 10 400 python -u bench.py --legs c3,c5 --no-cpu-baseline --steps 3 --warmup 1
echo "r04x done"
