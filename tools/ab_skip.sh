#!/bin/bash
# A/B of the MS-BFS slice activity skip on the C2 sweep and the C3 Clos sweep
# (GPU box, via gpurun, from the repo root): gpurun_out/$1/ab_skip.txt
set -e
TAG=${1:-ab}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
for SKIP in 1 0; do
  echo "ORH_MS_SKIP=$SKIP" >> "$OUT/ab_skip.txt"
  ORH_MS_SKIP=$SKIP timeout -k 10 300 python -u bench.py --scaling strong --steps 20 --warmup 3 \
    --no-cpu-baseline --no-route-db --legs '' >> "$OUT/ab_skip.txt" 2>> "$OUT/ab_skip.err"
done
