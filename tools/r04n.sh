#!/bin/bash
# Round-4 GPU pass n: the default bench line (N = 1, every leg, CPU baseline).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04n}
mkdir -p "$OUT"
timeout -k 10 1000 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench rc=$?" >> "$OUT/steps.txt"
