#!/bin/bash
# Targeted GPU pass: selected test files, then optional tools, each under its
# own time limit; stops at the first failure.
# usage (via gpurun): tools/gpu_check.sh TAG "tests/a.py tests/b.py" ["python tools/x.py ..."]...
set -e
TAG=$1
TESTS=$2
shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
fi
i=0
for CMD in "$@"; do
  i=$((i + 1))
  timeout -k 10 400 $CMD > "$OUT/cmd$i.out" 2> "$OUT/cmd$i.err"
done
echo "gpu_check $TAG done"
