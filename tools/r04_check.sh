#!/bin/bash
# Round-4 GPU pass: new policy tests first, the whole GPU suite, the C5 leg.
# usage (repo root, via gpurun): tools/r04_check.sh TAG [pytest -k expr]
set -e
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_wire.py -x -v --timeout 300 --timeout-method thread > "$OUT/policy_tests.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 600 python -u bench.py --legs c5 --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
echo "r04_check $TAG done"
