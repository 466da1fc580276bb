#!/bin/bash
# One GPU-box pass: gpu tests, smoke, default bench, kernel-trace stats.
# usage (from the repo root, via gpurun): tools/gpu_round.sh TAG
set -e
TAG=${1:-cur}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-route-db --legs '' --topologies 1 --lanes 1 > "$OUT/trace.log" 2>&1
echo "gpu_round $TAG done"
